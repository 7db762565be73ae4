#!/bin/bash
# head_bwd_w grid-cap sweep in the LSTM step (kernel-trace per variant)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp WELLFLOW_COOP=0
mkdir -p gpurun_out
for g in 512 256 128 64; do
  WELLFLOW_HEADW_GRID=$g timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/headw_$g -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/headw_$g.log 2>&1 || exit 1
done
