#!/bin/bash
# PMC counters for the LSTM training step kernels (counter collection only, no tracing domains)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
grep -oE "^\s*(SQ|TCC|TCP|GRBM|TA|TD)[A-Za-z0-9_]*" gpurun_out/pmc/counters_list.txt | sort -u | head -400 > gpurun_out/pmc/names.txt || true
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/set$i -o run -- python3 bench.py --steps 2 --warmup 1 --no-graph > gpurun_out/pmc/set$i.log 2>&1 || { echo "set $i failed"; tail -5 gpurun_out/pmc/set$i.log; exit 1; }
done
ls -R gpurun_out/pmc | head -40
