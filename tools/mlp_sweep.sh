#!/bin/bash
# MLP step variants (static bench): dW2 kernel vs stored-H1 GEMM, dW2 split depth
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "WELLFLOW_MLP_DW2=gemm" "WELLFLOW_MLP_DW2_SPLIT=32" "WELLFLOW_MLP_DW2_SPLIT=64" "WELLFLOW_MLP_DW2_SPLIT=128"; do
  echo "== $v"
  env $v timeout -k 10 120 python bench.py --model mlp --steps 30 --warmup 5 | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value']/1e6, r['ms_per_step'])" || exit $?
done
