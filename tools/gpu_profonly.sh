#!/bin/bash
# kernel-trace profiles of the three benches (plain launch of the persistent kernels)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
export WELLFLOW_COOP=0
for m in lstm mlp mlp_online; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$m -o run -- python3 bench.py --model $m --steps 20 --warmup 5 > gpurun_out/prof_$m.log 2>&1 || exit $?
  grep metric gpurun_out/prof_$m.log
done
