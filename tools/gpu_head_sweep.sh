#!/bin/bash
# head_fwd grid-cap sweep in the LSTM step (kernel-trace per variant)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp WELLFLOW_COOP=0
mkdir -p gpurun_out
for g in 2048 1024 512 256; do
  WELLFLOW_HEAD_GRID=$g timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/head_$g -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/head_$g.log 2>&1 || exit 1
  echo "grid=$g $(grep -h head_fwd gpurun_out/head_$g/run_kernel_stats.csv | cut -d, -f1-5)"
done
