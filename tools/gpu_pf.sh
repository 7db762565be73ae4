#!/bin/bash
# persistent-forward bring-up: its own test first (short limit), then the GPU tier, then bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 240 python -m pytest tests/test_kernels_gpu.py -q -x -k persistent > gpurun_out/pf.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/pf.log | tail -25
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -m pytest tests -q -x -m gpu > gpurun_out/tgpu.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/tgpu.log | tail -15
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 || exit $?
WELLFLOW_PERSISTENT=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 || exit $?
timeout -k 10 300 python tools/tune_lstm.py --rounds 3 --fwd 6 --bwd 8 --ksplit 16 > gpurun_out/tune_pf.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/tune_pf.log | tail -12
exit $rc
