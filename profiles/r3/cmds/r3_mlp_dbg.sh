#!/bin/bash
# MLP fixed-cost diagnosis: kernel times at 1 and 16 chunks per workgroup with the timing-only
# switches WELLFLOW_MLP_DBG = 0 (production), 1 (no epilogue atomics), 2 (no W2 loads), 3 (both)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for dbg in ${DBGS:-0 1 2 3}; do
  for b in 16384 262144; do
    WELLFLOW_MLP_DBG=$dbg timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/md_${dbg}_$b -o run \
      -- python3 bench.py --model mlp --batch $b --secondary none > gpurun_out/md_${dbg}_$b.log 2>&1 || exit $?
    echo "DBG=$dbg B=$b $(python3 tools/kstats.py gpurun_out/md_${dbg}_$b/run_kernel_stats.csv | grep -E 'mlp2' | awk '{printf "%s %s | ", $2, $(NF-2)}')"
  done
done
