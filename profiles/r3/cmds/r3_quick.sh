#!/bin/bash
# quick GPU check after a kernel edit: LSTM kernel/numerics tests, bench, kernel-trace stats
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_numerics_gpu.py ${EXTRA_TESTS} > gpurun_out/tq.log 2>&1; rc=$?
tail -3 gpurun_out/tq.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/tq.log; exit $rc; }
for i in 1 2; do timeout -k 10 200 python bench.py --secondary none > gpurun_out/bq$i.log 2>&1 || exit $?; python3 -c "import json,sys; r=json.loads([l for l in open('gpurun_out/bq$i.log') if l.startswith('{')][0]); print('bench', r['value'], r['ms_per_step'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_q -o run -- python3 bench.py --secondary none > gpurun_out/prof_q.log 2>&1 || exit $?
find gpurun_out/prof_q -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \;
