#!/bin/bash
# PMC table (3 passes: SQ / FETCH+TCC_HIT / WRITE+TCC_MISS, the r2 sets) of the LSTM step at the
# default dW tile and at WELLFLOW_DW_BIG=3 (round-2 tile), and of the static MLP step
set -o pipefail
export TMPDIR=/tmp
S1="GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES"
S2="GRBM_GUI_ACTIVE FETCH_SIZE TCC_HIT_sum"
S3="GRBM_GUI_ACTIVE WRITE_SIZE TCC_MISS_sum"
run_sets() {  # $1 = out dir, rest = bench args
  local out=$1; shift
  mkdir -p $out
  local i=0
  for set in "$S1" "$S2" "$S3"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $out/set$i -o run \
      -- python3 bench.py --steps 2 --warmup 1 --no-graph --secondary none "$@" > $out/set$i.log 2>&1 \
      || { tail -5 $out/set$i.log; return 1; }
  done
}
run_sets gpurun_out/pmc_dw7 || exit 1
python3 tools/pmc_table.py gpurun_out/pmc_dw7 persistent gemm_dw
WELLFLOW_DW_BIG=3 run_sets gpurun_out/pmc_dw3 || exit 1
python3 tools/pmc_table.py gpurun_out/pmc_dw3 gemm_dw
run_sets gpurun_out/pmc_mlp --model mlp --steps 3 || exit 1
python3 tools/pmc_table.py gpurun_out/pmc_mlp mlp2
