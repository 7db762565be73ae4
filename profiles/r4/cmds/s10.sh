# round 4, session 10: LSTM numerics after the fused head, full bench line, MLP phase timeline,
# then 8 more LSTM parity seeds
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u -m pytest tests/test_numerics_gpu.py tests/test_kernels_gpu.py tests/test_engines_gpu.py -v -m gpu \
  --timeout 200 --timeout-method thread -k "lstm or head" > gpurun_out/r4/s10_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r4/s10_tests.log | tail -2; grep -E "FAILED|ERROR" gpurun_out/r4/s10_tests.log | head
[ $rc -eq 0 ] || { tail -40 gpurun_out/r4/s10_tests.log; exit $rc; }
timeout -k 10 400 python bench.py > gpurun_out/r4/s10_bench.log 2>&1 || { tail -20 gpurun_out/r4/s10_bench.log; exit 1; }
grep '^{' gpurun_out/r4/s10_bench.log | cut -c1-400
timeout -k 10 300 python -u -m pytest tests/test_engines_gpu.py -v -m gpu --timeout 120 --timeout-method thread -k "mlp" \
  > gpurun_out/r4/s10_mlp_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r4/s10_mlp_tests.log | head; exit 1; }
grep -E "passed|failed" gpurun_out/r4/s10_mlp_tests.log | tail -1
for b4 in 0 1 0 1; do
  WELLFLOW_MLP_STEP_B4=$b4 timeout -k 10 200 python bench.py --model mlp --steps 300 --warmup 10 --secondary none --parity none \
    > gpurun_out/r4/mlp_b4_$b4.log 2>&1 || exit 1
  echo "B4=$b4 $(grep -o '"value": [0-9.]*' gpurun_out/r4/mlp_b4_$b4.log)"
done
WELLFLOW_MLP_STAMP=1 timeout -k 10 120 python -u tools/mlp_timeline.py > gpurun_out/r4/mlp_timeline.txt 2>&1 || { tail -20 gpurun_out/r4/mlp_timeline.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r4/mlp_timeline.txt
MODELS=lstm SEEDS=8,9,10,11,12,13,14,15 TAG=b TLIM=600 bash profiles/r4/cmds/s4.sh
