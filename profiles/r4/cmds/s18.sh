# round 4, session 18: PMC passes of the MLP step at HEAD (layer-2 read-ahead) and of the LSTM step (persistent fwd / bwd, dW GEMM with slab)
set -o pipefail
export TMPDIR=/tmp
S1="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
S2="GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_ADDR_CONFLICT"
S3="GRBM_GUI_ACTIVE FETCH_SIZE TCC_HIT_sum SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM SQ_LDS_UNALIGNED_STALL SQ_LDS_MEM_VIOLATIONS SQ_INSTS_LDS_ATOMIC"
S4="GRBM_GUI_ACTIVE WRITE_SIZE TCC_MISS_sum SQ_WAVES SQ_INSTS_BRANCH SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL"
out=gpurun_out/r4/pmc_mlp5; mkdir -p $out; i=0
for set in "$S1" "$S2" "$S3" "$S4"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $out/set$i -o run \
    -- python3 bench.py --model mlp --steps 3 --warmup 1 --no-graph --secondary none --parity none > $out/set$i.log 2>&1 \
    || { tail -5 $out/set$i.log; exit 1; }
done
python3 tools/pmc_table.py $out mlp2 adam > $out/pmc_table.md; cat $out/pmc_table.md
out=gpurun_out/r4/pmc_lstm; mkdir -p $out; i=0
for set in "$S1" "$S2" "$S3" "$S4"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $out/set$i -o run \
    -- python3 bench.py --steps 3 --warmup 1 --no-graph --secondary none --parity none > $out/set$i.log 2>&1 \
    || { tail -5 $out/set$i.log; exit 1; }
done
python3 tools/pmc_table.py $out lstm_ gemm_dw dw_slab > $out/pmc_table.md; cat $out/pmc_table.md
python3 - <<'PY'
import csv, glob, collections
v = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/r4/pmc_mlp5/set*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "mlp2_step" in r["Kernel_Name"] or "dw2f" in r["Kernel_Name"]:
            v[r["Kernel_Name"].split("(")[0][-30:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in v.items():
    print(k, {n: f"{sum(x)/len(x):.4g}" for n, x in sorted(c.items())})
PY
