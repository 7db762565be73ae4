#!/bin/bash
# MLP kernel time vs rows per workgroup (fixed prologue cost vs per-chunk cost): kernel-trace
# stats of bench.py --model mlp at B = 16384 .. 262144 (1 .. 16 64-row chunks per workgroup)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in ${BATCHES:-16384 32768 65536 131072 262144}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mlps_$b -o run \
    -- python3 bench.py --model mlp --batch $b --secondary none > gpurun_out/mlps_$b.log 2>&1 || exit $?
  echo "B=$b $(grep -o '"value": [0-9.]*' gpurun_out/mlps_$b.log | head -1)"
  python3 tools/kstats.py gpurun_out/mlps_$b/run_kernel_stats.csv | grep -E "mlp2|adam" | cut -c1-40,89-
done
