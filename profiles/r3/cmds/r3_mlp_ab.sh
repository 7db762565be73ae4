#!/bin/bash
# MLP forward A/B: production vs H1 fragments double-buffered (WELLFLOW_MLP_DBG=4) vs setprio
# clusters (WELLFLOW_MLP_PRIO=1), interleaved kernel-trace runs; MLP GPU tests first
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_engines_gpu.py tests/test_numerics_gpu.py > gpurun_out/tmlp.log 2>&1; rc=$?
tail -2 gpurun_out/tmlp.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/tmlp.log; exit $rc; }
i=0
for arm in "WELLFLOW_MLP_DBG=0" "WELLFLOW_MLP_DBG=4" "WELLFLOW_MLP_PRIO=1" "WELLFLOW_MLP_DBG=0" "WELLFLOW_MLP_DBG=4" "WELLFLOW_MLP_PRIO=1"; do
  i=$((i+1))
  env $arm timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mab_$i -o run \
    -- python3 bench.py --model mlp --secondary none > gpurun_out/mab_$i.log 2>&1 || exit $?
  echo "$arm $(grep -o '"value": [0-9.]*' gpurun_out/mab_$i.log | head -1) $(python3 tools/kstats.py gpurun_out/mab_$i/run_kernel_stats.csv | grep -E 'fwd_train' | awk '{print $(NF-2), $(NF-1)}')"
done
BATCHES="16384 262144" bash tools/r3_mlp_scan.sh
