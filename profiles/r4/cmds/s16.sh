# round 4, session 16: LSTM dW GEMM split-K partials as plain-stored slab + one reduce (vs fp32 atomics)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_numerics_gpu.py tests/test_determinism_gpu.py \
  tests/test_step_gpu.py tests/test_dp_native_gpu.py tests/test_torch_ops_gpu.py -v -m gpu \
  --timeout 120 --timeout-method thread -k "lstm" > gpurun_out/r4/s16_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r4/s16_tests.log | tail -1; grep -E "FAILED|Error" gpurun_out/r4/s16_tests.log | head
[ $rc -eq 0 ] || { tail -40 gpurun_out/r4/s16_tests.log; exit $rc; }
for cfg in 1 0 1 0; do
  WELLFLOW_DW_SLAB=$cfg timeout -k 10 200 python bench.py --steps 60 --warmup 5 --secondary none --parity none \
    > gpurun_out/r4/lstm_s16_$cfg.log 2>&1 || { tail -20 gpurun_out/r4/lstm_s16_$cfg.log; exit 1; }
  echo "SLAB=$cfg $(grep -o '"value": [0-9.]*, "unit": "rows/s", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/r4/lstm_s16_$cfg.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_lstm16 -o run \
  -- python3 bench.py --steps 20 --warmup 3 --secondary none --parity none > gpurun_out/r4/prof_lstm16.log 2>&1 || { tail -30 gpurun_out/r4/prof_lstm16.log; exit 1; }
find gpurun_out/r4/prof_lstm16 -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \;
