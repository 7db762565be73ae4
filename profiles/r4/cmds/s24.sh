# round 4, session 24: CNN forward/backward kernels, static s_setprio 1 for waves 4-7 (WELLFLOW_CNN_PRIO) A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
WELLFLOW_CNN_PRIO=1 timeout -k 10 300 python -u -m pytest tests/ -v -m gpu \
  --timeout 120 --timeout-method thread -k "cnn" > gpurun_out/r4/s24_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r4/s24_tests.log | tail -1
[ $rc -eq 0 ] || { tail -40 gpurun_out/r4/s24_tests.log; exit $rc; }
for cfg in 1 0 1 0 1 0; do
  WELLFLOW_CNN_PRIO=$cfg timeout -k 10 200 python bench.py --model cnn --steps 600 --warmup 10 --secondary none --parity none \
    > gpurun_out/r4/cnn_s24_$cfg.log 2>&1 || { tail -20 gpurun_out/r4/cnn_s24_$cfg.log; exit 1; }
  echo "CNN_PRIO=$cfg $(grep -o '"value": [0-9.]*, "unit": "[a-z/]*", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/r4/cnn_s24_$cfg.log)"
done
for cfg in 0 1; do
  WELLFLOW_CNN_PRIO=$cfg timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_cnn24_$cfg -o run \
    -- python3 bench.py --model cnn --steps 100 --warmup 5 --secondary none --parity none > gpurun_out/r4/prof_cnn24_$cfg.log 2>&1 || { tail -30 gpurun_out/r4/prof_cnn24_$cfg.log; exit 1; }
  echo "CNN_PRIO=$cfg"; find gpurun_out/r4/prof_cnn24_$cfg -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \; | head -3
done
