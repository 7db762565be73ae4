#!/bin/bash
# LSTM step: Adam grid cap A/B (WELLFLOW_ADAM_GRID) under kernel trace, LSTM GPU tests first
set -o pipefail
export TMPDIR=/tmp
VAR=WELLFLOW_ADAM_GRID VALS="${VALS:-256 2048 256 2048}" KERN="adam|persistent|dw" bash tools/r3_ab.sh
