#!/bin/bash
# A/B of a production-correct kernel variant in ONE box: tests first, then interleaved
# kernel-trace runs of bench.py per value of VAR (default WELLFLOW_PF_DBG "0 4096 0 4096")
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
VAR=${VAR:-WELLFLOW_PF_DBG}; VALS=${VALS:-"0 4096 0 4096"}; KERN=${KERN:-persistent}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_numerics_gpu.py > gpurun_out/tab.log 2>&1; rc=$?
tail -2 gpurun_out/tab.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/tab.log; exit $rc; }
i=0
for v in $VALS; do
  i=$((i+1))
  env "$VAR=$v" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_$i -o run \
    -- python3 bench.py --secondary none ${BENCH_ARGS} > gpurun_out/ab_$i.log 2>&1 || exit $?
  b=$(python3 -c "import json; r=json.loads([l for l in open('gpurun_out/ab_$i.log') if l.startswith('{')][0]); print(r['value'], r['ms_per_step'])")
  echo "$VAR=$v bench $b"
  python3 tools/kstats.py gpurun_out/ab_$i/run_kernel_stats.csv | grep -E "$KERN" | cut -c1-40,89-
done
