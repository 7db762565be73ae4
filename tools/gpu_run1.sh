#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -rf > gpurun_out/t1.log 2>&1; rc=$?
tail -30 gpurun_out/t1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc, stopping"; exit $rc; fi
timeout -k 10 300 python __graft_entry__.py smoke || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch 4096 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch 8192 || exit $?
