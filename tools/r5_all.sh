# round-5 GPU pass: selected tests (TF, a run_sel.py file), then one kernel-trace profile per
# model in MODELS (bench.py, 20 steps), then the default bench line. Each GPU step has its own
# limit; the chain stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
if [ -n "$TF" ]; then
  timeout -k 10 ${TT:-600} python -u tools/run_sel.py $TF -x -v --timeout 120 --timeout-method thread > gpurun_out/r5/t.log 2>&1; rc=$?
  grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r5/t.log | tail -60
  [ $rc -ne 0 ] && { tail -40 gpurun_out/r5/t.log; exit $rc; }
fi
for m in $MODELS; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/prof_${TAG}_$m -o run \
    -- python3 bench.py --model $m --secondary none --parity none --steps ${PSTEPS:-20} --warmup 3 > gpurun_out/r5/prof_${TAG}_$m.log 2>&1 || exit $?
  find gpurun_out/r5/prof_${TAG}_$m -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \; | head -10
  tail -1 gpurun_out/r5/prof_${TAG}_$m.log | cut -c1-200
done
if [ -n "$BENCH" ]; then
  timeout -k 10 500 python -u bench.py $BENCH > gpurun_out/r5/bench_$TAG.log 2>&1; rc=$?
  tail -1 gpurun_out/r5/bench_$TAG.log | cut -c1-1500
  exit $rc
fi
