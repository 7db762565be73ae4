# round 4, session 22: LSTM dW GEMM (256x288), per-cluster s_setprio (1) vs static priority for waves 4-7 (3)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
WELLFLOW_DW288_PRIO=3 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -v -m gpu \
  --timeout 120 --timeout-method thread -k "lstm or weight_gradient" > gpurun_out/r4/s22_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r4/s22_tests.log | tail -1
[ $rc -eq 0 ] || { tail -40 gpurun_out/r4/s22_tests.log; exit $rc; }
for cfg in 3 1 3 1 3 1; do
  WELLFLOW_DW288_PRIO=$cfg timeout -k 10 200 python bench.py --steps 100 --warmup 5 --secondary none --parity none \
    > gpurun_out/r4/lstm_s22_$cfg.log 2>&1 || { tail -20 gpurun_out/r4/lstm_s22_$cfg.log; exit 1; }
  echo "DW288_PRIO=$cfg $(grep -o '"value": [0-9.]*, "unit": "rows/s", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/r4/lstm_s22_$cfg.log)"
done
for cfg in 1 3; do
  WELLFLOW_DW288_PRIO=$cfg timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_lstm22_$cfg -o run \
    -- python3 bench.py --steps 20 --warmup 3 --secondary none --parity none > gpurun_out/r4/prof_lstm22_$cfg.log 2>&1 || { tail -30 gpurun_out/r4/prof_lstm22_$cfg.log; exit 1; }
  echo "DW288_PRIO=$cfg"; find gpurun_out/r4/prof_lstm22_$cfg -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \; | head -4
done
