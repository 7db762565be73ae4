#!/bin/bash
# tests first (stop on any crash), then the variant tuner
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py tests/test_engines_gpu.py -q -x -m gpu > gpurun_out/t3.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/t3.log | tail -15
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python tools/tune_lstm.py "$@" > gpurun_out/tune.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/tune.log
exit $rc
