#!/bin/bash
# LSTM run-to-run variance: N separate bench processes under a kernel trace; per run the bench
# value and the mean duration of the three big kernels (fwd / bwd persistent, dW GEMM).
set -o pipefail
O=${1:-gpurun_out/r5/lstmvar}; N=${2:-5}
mkdir -p $O; export TMPDIR=/tmp
for i in $(seq 1 $N); do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/r$i -o run -- python3 bench.py --secondary none --parity none --steps 40 > $O/r$i.log 2>&1 || exit 1
  f=$(find $O/r$i -name "*kernel_trace.csv" | head -1)
  python3 - "$f" "$O/r$i.log" <<'PY'
import csv, json, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    for k in ("lstm_fwd_persistent", "lstm_bwd_persistent", "gemm_dw_h"):
        if k in n:
            d[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
v = [json.loads(l)["value"] for l in open(sys.argv[2]) if l.startswith("{")]
print(round(v[-1] / 1e6, 4) if v else None, {k: round(sum(x[-30:]) / len(x[-30:]) / 1e3, 1) for k, x in d.items()}, flush=True)
PY
  rm -rf $O/r$i
done
