#!/bin/bash
# full GPU test tier, then the headline bench with and without hipGraph capture
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -x -m gpu > gpurun_out/tgpu.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/tgpu.log | tail -15
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py "$@" || exit $?
timeout -k 10 300 python bench.py --no-graph "$@" || exit $?
timeout -k 10 300 python bench.py "$@" || exit $?
