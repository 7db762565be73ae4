#!/bin/bash
# GPU tier + MLP benches (static / online), each step time-limited, first failure ends the call
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/tgpu.log 2>&1; rc=$?
grep -E "passed|failed|error" gpurun_out/tgpu.log | tail -5
[ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" gpurun_out/tgpu.log | tail -60; exit $rc; }
timeout -k 10 300 python bench.py --model mlp || exit $?
timeout -k 10 300 python bench.py --model mlp_online || exit $?
WELLFLOW_MLP_MASK=0 timeout -k 10 300 python bench.py --model mlp || exit $?
