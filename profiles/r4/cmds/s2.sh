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
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
  > gpurun_out/r4/s2_tests.log 2>&1; rc=$?
grep -E "passed|failed|error" gpurun_out/r4/s2_tests.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/r4/s2_tests.log | head -20; tail -80 gpurun_out/r4/s2_tests.log; exit $rc; }
timeout -k 10 300 python __graft_entry__.py smoke || exit $?
timeout -k 10 400 python bench.py > gpurun_out/r4/s2_bench.log 2>&1 || { tail -20 gpurun_out/r4/s2_bench.log; exit 1; }
grep '^{' gpurun_out/r4/s2_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_cnn -o run \
  -- python3 bench.py --model cnn --steps 50 --warmup 5 > gpurun_out/r4/prof_cnn.log 2>&1 || { tail -30 gpurun_out/r4/prof_cnn.log; exit 1; }
find gpurun_out/r4/prof_cnn -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_lstm -o run \
  -- python3 bench.py --secondary none --parity none > gpurun_out/r4/prof_lstm.log 2>&1 || { tail -30 gpurun_out/r4/prof_lstm.log; exit 1; }
find gpurun_out/r4/prof_lstm -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_mlp -o run \
  -- python3 bench.py --model mlp --steps 50 --warmup 5 > gpurun_out/r4/prof_mlp.log 2>&1 || { tail -30 gpurun_out/r4/prof_mlp.log; exit 1; }
find gpurun_out/r4/prof_mlp -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \;
