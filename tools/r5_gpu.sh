# round-5 GPU helper: optional pytest selection (T="file::expr" or "file -k expr"), then optional
# kernel trace (P=tag) of the LSTM bench. Every GPU step has its own limit; chained.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
if [ -n "$TF" ]; then
  timeout -k 10 600 python -u tools/run_sel.py $TF -x -v --timeout 120 --timeout-method thread > gpurun_out/r5/t.log 2>&1; rc=$?
  grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r5/t.log | tail -40
  [ $rc -ne 0 ] && { tail -40 gpurun_out/r5/t.log; exit $rc; }
fi
if [ -n "$T" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread $T > gpurun_out/r5/t.log 2>&1; rc=$?
  grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r5/t.log | tail -40
  [ $rc -ne 0 ] && { tail -40 gpurun_out/r5/t.log; exit $rc; }
fi
if [ -n "$P" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/prof_$P -o run \
    -- python3 bench.py --secondary none --parity none --steps 20 --warmup 3 $BARGS > gpurun_out/r5/prof_$P.log 2>&1 || exit $?
  find gpurun_out/r5/prof_$P -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \; | head -8
fi
if [ -n "$B" ]; then
  timeout -k 10 400 python -u bench.py $B > gpurun_out/r5/bench.log 2>&1; rc=$?
  tail -1 gpurun_out/r5/bench.log | cut -c1-400
  exit $rc
fi
