#!/bin/bash
# H2D stall investigation (tools/h2d_stall.py): queue-ordered vs host-ordered slot refills,
# the SDMA-off variant, and one traced run (kernel + memory-copy trace) of the queue mode
export TMPDIR=/tmp
mkdir -p gpurun_out/h2d
set -o pipefail
for m in queue host; do
  timeout -k 10 120 python tools/h2d_stall.py --mode $m --out gpurun_out/h2d/$m.json || exit $?
done
HSA_ENABLE_SDMA=0 timeout -k 10 120 python tools/h2d_stall.py --mode queue --out gpurun_out/h2d/queue_nosdma.json || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/h2d/trace -o run \
  -- python3 tools/h2d_stall.py --mode queue --iters 200 --out gpurun_out/h2d/queue_traced.json > gpurun_out/h2d/trace.log 2>&1 || exit $?
tail -1 gpurun_out/h2d/trace.log
ls gpurun_out/h2d/trace
