# round 4, session 2: the whole GPU test tier (fused CNN, bf16 cell-state history, diag
# switches, DP pre-flight, parity), bench.py, then kernel traces of the CNN and LSTM benches.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
for a in "1 527 8" "0 528 8" "4 528 8" "1 528 8"; do
  timeout -k 10 60 tools/memset_repro.bin $a >> gpurun_out/r4/memset_repro.log 2>&1; r=$?
  [ $r -le 1 ] || { echo "memset repro rc=$r"; exit $r; }
done
grep RESULT gpurun_out/r4/memset_repro.log
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread \
  > gpurun_out/r4/s2_tests.log 2>&1; rc=$?
grep -E "passed|failed|error" gpurun_out/r4/s2_tests.log | tail -3
grep -E "FAILED|ERROR" gpurun_out/r4/s2_tests.log | head -20
# 1 = some tests failed (keep measuring); anything else (crash, abort, time limit) ends the call
[ $rc -le 1 ] || { tail -60 gpurun_out/r4/s2_tests.log; exit $rc; }
timeout -k 10 300 python __graft_entry__.py smoke || exit $?
timeout -k 10 400 python bench.py > gpurun_out/r4/s2_bench.log 2>&1 || { tail -20 gpurun_out/r4/s2_bench.log; exit 1; }
grep '^{' gpurun_out/r4/s2_bench.log
