#!/bin/bash
# PMC counters for the static-MLP training step kernels (counter collection only, one pass per set)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_mlp
i=0
for set in "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES" "FETCH_SIZE TCC_HIT_sum" "TCC_MISS_sum WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_mlp/set$i -o run -- python3 bench.py --model mlp --steps 2 --warmup 1 --no-graph > gpurun_out/pmc_mlp/set$i.log 2>&1 || { echo "set $i failed"; tail -5 gpurun_out/pmc_mlp/set$i.log; exit 1; }
done
find gpurun_out/pmc_mlp -name "*counter_collection.csv"
