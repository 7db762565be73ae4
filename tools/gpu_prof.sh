#!/bin/bash
# usage: bash tools/gpu_prof.sh <outdir-name> [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
name=$1; shift
mkdir -p gpurun_out/$name
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$name -o run -- python3 bench.py "$@" > gpurun_out/$name/bench.log 2>&1
rc=$?
tail -5 gpurun_out/$name/bench.log
find gpurun_out/$name -name "*kernel_stats.csv" | head -3
exit $rc
