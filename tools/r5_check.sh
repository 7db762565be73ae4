# round-5 quick GPU check: LSTM persistent tests + numerics + bench (each step time-limited, chained)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "persistent" tests/test_numerics_gpu.py > gpurun_out/r5/t_lstm.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r5/t_lstm.log | tail -30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --secondary none --parity none > gpurun_out/r5/bench.log 2>&1; rc=$?
tail -3 gpurun_out/r5/bench.log
exit $rc
