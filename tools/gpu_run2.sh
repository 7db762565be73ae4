#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py tests/test_engines_gpu.py -q -rf -m gpu > gpurun_out/t2.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/t2.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc, stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 || exit $?
