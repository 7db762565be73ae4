# round 4, session 25: the whole GPU test tier at HEAD (final, after the CNN priority knob), smoke, the bench line, kernel traces
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread \
  > gpurun_out/r4/final4_tests.log 2>&1; rc=$?
grep -E "passed|failed|error" gpurun_out/r4/final4_tests.log | tail -2
grep -E "FAILED|ERROR" gpurun_out/r4/final4_tests.log | head -20
[ $rc -le 1 ] || { tail -60 gpurun_out/r4/final4_tests.log; exit $rc; }
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/r4/final4_smoke.log 2>&1 || { tail -20 gpurun_out/r4/final4_smoke.log; exit 1; }
tail -1 gpurun_out/r4/final4_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r4/final4_bench.log 2>&1 || { tail -20 gpurun_out/r4/final4_bench.log; exit 1; }
grep '^{' gpurun_out/r4/final4_bench.log | cut -c1-300
