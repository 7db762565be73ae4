#!/bin/bash
# rocprofv3 counter list + PMC passes over a 2-step LSTM bench (no graph): one pass per set
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc3
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc3/counters.txt 2>&1 || true
i=0
for set in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS" \
           "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc3/set$i -o run \
    -- python3 bench.py --steps 2 --warmup 1 --no-graph --secondary none ${PMC_ARGS} > gpurun_out/pmc3/set$i.log 2>&1 || { tail -5 gpurun_out/pmc3/set$i.log; exit 1; }
done
python3 tools/pmc_table.py gpurun_out/pmc3 persistent gemm_dw
