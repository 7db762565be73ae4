#!/bin/bash
# GPU tier + all three benches, each step time-limited, first failure ends the call
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/tgpu.log 2>&1; rc=$?
grep -E "passed|failed|error" gpurun_out/tgpu.log | tail -5
[ $rc -ne 0 ] && { grep -B5 -A40 "FAILED\|Error" gpurun_out/tgpu.log | tail -60; exit $rc; }
timeout -k 10 300 python __graft_entry__.py smoke || exit $?
for m in mlp mlp_online lstm; do timeout -k 10 300 python bench.py --model $m || exit $?; done
