# round 4, session 5: MLP A/B (one-launch step / fragment dW2 / the round-3 pair) + kernel trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
for cfg in "1 1" "1 0" "0 0"; do
  set -- $cfg
  WELLFLOW_MLP_STEP=$1 WELLFLOW_MLP_DW2F=$2 timeout -k 10 200 python bench.py --model mlp --steps 300 --warmup 10 --secondary none --parity none \
    > gpurun_out/r4/mlp_ab_$1$2.log 2>&1 || { tail -20 gpurun_out/r4/mlp_ab_$1$2.log; exit 1; }
  echo "STEP=$1 DW2F=$2 $(grep -o '"value": [0-9.]*, "unit": "rows/s", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/r4/mlp_ab_$1$2.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_mlp -o run \
  -- python3 bench.py --model mlp --steps 50 --warmup 5 --secondary none --parity none > gpurun_out/r4/prof_mlp.log 2>&1 || { tail -30 gpurun_out/r4/prof_mlp.log; exit 1; }
find gpurun_out/r4/prof_mlp -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \;
