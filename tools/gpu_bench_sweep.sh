#!/bin/bash
# bench.py under several option sets, one line each: tools/gpu_bench_sweep.sh "<opts1>" "<opts2>" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for o in "$@"; do
  echo "== $o"
  timeout -k 10 240 python bench.py --steps 30 --warmup 5 $o > gpurun_out/sweep.log 2>&1 || { tail -20 gpurun_out/sweep.log; exit 1; }
  grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*' gpurun_out/sweep.log | tr '\n' ' '; echo
done
