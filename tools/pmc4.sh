# Four rocprofv3 --pmc passes (<= 8 SQ, <= 4 TCC counters each) over a short ungraphed bench
# run of one model, then the per-kernel table (tools/pmc_table.py).
#   tools/pmc4.sh OUTDIR MODEL "kernel-substrings" [extra bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=$1; model=$2; filt=$3; shift 3
S1="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
S2="GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_ADDR_CONFLICT"
S3="GRBM_GUI_ACTIVE FETCH_SIZE TCC_HIT_sum SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM SQ_LDS_UNALIGNED_STALL SQ_LDS_MEM_VIOLATIONS SQ_INSTS_LDS_ATOMIC"
S4="GRBM_GUI_ACTIVE WRITE_SIZE TCC_MISS_sum SQ_WAVES SQ_INSTS_BRANCH SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL"
mkdir -p $out; i=0
for set in "$S1" "$S2" "$S3" "$S4"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $out/set$i -o run \
    -- python3 bench.py --model $model --steps 3 --warmup 1 --no-graph --secondary none --parity none "$@" > $out/set$i.log 2>&1 \
    || { tail -5 $out/set$i.log; exit 1; }
done
python3 tools/pmc_table.py $out $filt > $out/pmc_table.md; cat $out/pmc_table.md
