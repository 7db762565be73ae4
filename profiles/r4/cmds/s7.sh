# round 4, session 7: MLP numerics (one-launch step + dW2F vs the pair) then the A/B bench + kernel trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_engines_gpu.py -v -m gpu --timeout 120 --timeout-method thread -k "mlp" \
  > gpurun_out/r4/s7_tests.log 2>&1; rc=$?
grep -E "passed|failed|error" gpurun_out/r4/s7_tests.log | tail -2; grep -E "FAILED|ERROR" gpurun_out/r4/s7_tests.log | head
[ $rc -le 1 ] || { tail -40 gpurun_out/r4/s7_tests.log; exit $rc; }
bash profiles/r4/cmds/s5.sh
