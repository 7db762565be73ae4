#!/bin/bash
# PMC table (3 passes, the r2 sets) of the static MLP step
set -o pipefail
export TMPDIR=/tmp
S1="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES"
S2="GRBM_GUI_ACTIVE FETCH_SIZE TCC_HIT_sum"
S3="GRBM_GUI_ACTIVE WRITE_SIZE TCC_MISS_sum"
out=gpurun_out/pmc_mlp2; mkdir -p $out; i=0
for set in "$S1" "$S2" "$S3"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $out/set$i -o run \
    -- python3 bench.py --model mlp --steps 3 --warmup 1 --no-graph --secondary none > $out/set$i.log 2>&1 \
    || { tail -5 $out/set$i.log; exit 1; }
done
python3 tools/pmc_table.py $out mlp2
