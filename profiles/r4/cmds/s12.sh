# round 4, session 12: final validation (s11) then the MLP barrier A/B, the MLP phase timeline
# and 8 more LSTM parity seeds
set -o pipefail
export TMPDIR=/tmp
bash profiles/r4/cmds/s11.sh || exit $?
for b4 in 0 1 0 1; do
  WELLFLOW_MLP_STEP_B4=$b4 timeout -k 10 200 python bench.py --model mlp --steps 300 --warmup 10 --secondary none --parity none \
    > gpurun_out/r4/mlp_b4_$b4.log 2>&1 || exit 1
  echo "B4=$b4 $(grep -o '"value": [0-9.]*' gpurun_out/r4/mlp_b4_$b4.log)"
done
WELLFLOW_MLP_STAMP=1 timeout -k 10 120 python -u tools/mlp_timeline.py > gpurun_out/r4/mlp_timeline.txt 2>&1 || { tail -20 gpurun_out/r4/mlp_timeline.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r4/mlp_timeline.txt
MODELS=lstm SEEDS=8,9,10,11,12,13,14,15 TAG=b TLIM=500 bash profiles/r4/cmds/s4.sh
