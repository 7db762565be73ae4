#!/bin/bash
# GPU tier + smoke + headline bench + kernel-trace profile; every GPU step time-limited,
# chained so the first failure ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/tgpu.log 2>&1; rc=$?
grep -E "passed|failed|error" gpurun_out/tgpu.log | tail -5
[ $rc -ne 0 ] && { tail -40 gpurun_out/tgpu.log; exit $rc; }
timeout -k 10 300 python __graft_entry__.py smoke || exit $?
timeout -k 10 300 python bench.py || exit $?
timeout -k 10 300 python bench.py --model mlp || exit $?
timeout -k 10 300 python bench.py --model mlp_online || exit $?
if [ "$1" = "prof" ]; then
  # rocprofv3 7.2 segfaults at exit after tracing a cooperative dispatch: plain launch
  export WELLFLOW_COOP=0
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_full -o run -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_full.log 2>&1 || exit $?
  find gpurun_out/prof_full -name "*kernel_stats.csv"
fi
if [ "$1" = "prof" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mlp -o run -- python3 bench.py --model mlp --steps 20 --warmup 5 > gpurun_out/prof_mlp.log 2>&1 || exit $?
  find gpurun_out/prof_mlp -name "*kernel_stats.csv"
fi
