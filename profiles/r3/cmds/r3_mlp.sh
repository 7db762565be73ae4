#!/bin/bash
# MLP GPU check: MLP / engine / numerics GPU tests, the kernel-time scan over the batch, and
# bench A/B of the spread reduction (WELLFLOW_MLP_SPREAD=1/0, interleaved)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_engines_gpu.py tests/test_numerics_gpu.py tests/test_step_gpu.py tests/test_torch_ops_gpu.py \
  > gpurun_out/tmlp.log 2>&1; rc=$?
tail -3 gpurun_out/tmlp.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/tmlp.log; exit $rc; }
BATCHES="${BATCHES:-16384 262144}" bash tools/r3_mlp_scan.sh || exit $?
for sp in 1 0 1 0; do
  for m in mlp mlp_online; do
    WELLFLOW_MLP_SPREAD=$sp timeout -k 10 200 python bench.py --model $m --secondary none > gpurun_out/mab.log 2>&1 || { tail -5 gpurun_out/mab.log; exit 1; }
    echo "SPREAD=$sp $m $(grep -o '"value": [0-9.]*, "unit": "[a-z/]*", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/mab.log)"
  done
done
