# round 4, session 21: MLP dW2F kernel, LDS fragments read a half-chunk ahead (WELLFLOW_DW2F_PF) A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_engines_gpu.py -v -m gpu \
  --timeout 120 --timeout-method thread -k "mlp" > gpurun_out/r4/s21_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r4/s21_tests.log | tail -1
[ $rc -eq 0 ] || { tail -40 gpurun_out/r4/s21_tests.log; exit $rc; }
for cfg in 1 0 1 0 1 0; do
  WELLFLOW_DW2F_PF=$cfg timeout -k 10 200 python bench.py --model mlp --steps 600 --warmup 10 --secondary none --parity none \
    > gpurun_out/r4/mlp_s21_$cfg.log 2>&1 || { tail -20 gpurun_out/r4/mlp_s21_$cfg.log; exit 1; }
  echo "DW2F_PF=$cfg $(grep -o '"value": [0-9.]*, "unit": "rows/s", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/r4/mlp_s21_$cfg.log)"
done
WELLFLOW_MLP_STAMP=1 timeout -k 10 120 python -u tools/mlp_timeline.py > gpurun_out/r4/mlp_timeline21.txt 2>&1 || { tail -20 gpurun_out/r4/mlp_timeline21.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r4/mlp_timeline21.txt
for cfg in 0 1; do
  WELLFLOW_DW2F_PF=$cfg timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_mlp21_$cfg -o run \
    -- python3 bench.py --model mlp --steps 100 --warmup 5 --secondary none --parity none > gpurun_out/r4/prof_mlp21_$cfg.log 2>&1 || { tail -30 gpurun_out/r4/prof_mlp21_$cfg.log; exit 1; }
  echo "DW2F_PF=$cfg"; find gpurun_out/r4/prof_mlp21_$cfg -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \; | head -5
done
