#!/bin/bash
# Baseline GPU pass at a checkpoint: full GPU test tier, smoke, bench.py (headline + secondaries),
# kernel-trace stats of the headline. Each GPU step has its own limit; the first failure ends it.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/tgpu.log 2>&1; rc=$?
tail -3 gpurun_out/tgpu.log; [ $rc -eq 0 ] || { tail -60 gpurun_out/tgpu.log; exit $rc; }
timeout -k 10 300 python __graft_entry__.py smoke || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
grep '^{' gpurun_out/bench_full.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_base -o run \
  -- python3 bench.py --secondary none > gpurun_out/prof_base.log 2>&1 || exit $?
find gpurun_out/prof_base -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \;
