#!/bin/bash
# dW2 GEMM sweep for the static MLP bench: tile x split-K depth
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for cfg in "0 0" "0 64" "0 128" "1 32" "1 64" "1 128" "1 256"; do
  set -- $cfg
  echo "tile=$1 ksplit=$2"
  WELLFLOW_MLP_DW_TILE=$1 WELLFLOW_MLP_DW_KSPLIT=$2 timeout -k 10 120 python bench.py --model mlp --steps 50 --warmup 10 | cut -c1-200 || exit $?
done
