# round 4, session 15: MLP step with layer-2 H1 fragment reads one K step ahead: numerics, A/B, trace, timeline
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_engines_gpu.py tests/test_dp_native_gpu.py tests/test_numerics_gpu.py -v -m gpu \
  --timeout 120 --timeout-method thread -k "mlp" > gpurun_out/r4/s15_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r4/s15_tests.log | tail -1; grep -E "FAILED|Error" gpurun_out/r4/s15_tests.log | head
[ $rc -eq 0 ] || { tail -40 gpurun_out/r4/s15_tests.log; exit $rc; }
for cfg in 1 0 1 0; do
  WELLFLOW_MLP_STEP=$cfg timeout -k 10 200 python bench.py --model mlp --steps 300 --warmup 10 --secondary none --parity none \
    > gpurun_out/r4/mlp_s15_$cfg.log 2>&1 || { tail -20 gpurun_out/r4/mlp_s15_$cfg.log; exit 1; }
  echo "STEP=$cfg $(grep -o '"value": [0-9.]*, "unit": "rows/s", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/r4/mlp_s15_$cfg.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_mlp15 -o run \
  -- python3 bench.py --model mlp --steps 50 --warmup 5 --secondary none --parity none > gpurun_out/r4/prof_mlp15.log 2>&1 || { tail -30 gpurun_out/r4/prof_mlp15.log; exit 1; }
find gpurun_out/r4/prof_mlp15 -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \;
WELLFLOW_MLP_STAMP=1 timeout -k 10 120 python -u tools/mlp_timeline.py > gpurun_out/r4/mlp_timeline15.txt 2>&1 || { tail -20 gpurun_out/r4/mlp_timeline15.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r4/mlp_timeline15.txt
