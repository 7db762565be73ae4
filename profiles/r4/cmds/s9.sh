# round 4, session 9: MLP step phase timeline (WELLFLOW_MLP_STAMP), then
# 8 more LSTM parity seeds (same numerics as production: no diagnostic switch is set)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
WELLFLOW_MLP_STAMP=1 timeout -k 10 120 python -u tools/mlp_timeline.py > gpurun_out/r4/mlp_timeline.txt 2>&1 || { tail -20 gpurun_out/r4/mlp_timeline.txt; exit 1; }
cat gpurun_out/r4/mlp_timeline.txt | grep -v amdgpu.ids
MODELS=lstm SEEDS=8,9,10,11,12,13,14,15 TAG=b TLIM=900 bash profiles/r4/cmds/s4.sh
