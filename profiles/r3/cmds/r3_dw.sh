#!/bin/bash
# dW tile A/B: standalone tile timings (tools/dw_tiles.py), then interleaved kernel-trace bench runs
# per WELLFLOW_DW_BIG value (tools/r3_ab.sh), dW / LSTM GPU tests first
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/dw_tiles.py ${TILES:-3 4 5} > gpurun_out/dw_tiles.log 2>&1; rc=$?
cat gpurun_out/dw_tiles.log; [ $rc -eq 0 ] || exit $rc
VAR=WELLFLOW_DW_BIG VALS="${VALS:-3 4 3 4}" KERN="dw|persistent" bash tools/r3_ab.sh
