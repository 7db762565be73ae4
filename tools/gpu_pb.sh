#!/bin/bash
# persistent-backward bring-up: numerics first, then the headline bench with it on / off
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "persistent_backward or lstm_forward_backward" --timeout 120 --timeout-method thread > gpurun_out/tpb.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|assert" gpurun_out/tpb.log | head -30
[ $rc -ne 0 ] && { tail -30 gpurun_out/tpb.log; exit $rc; }
timeout -k 10 300 python bench.py || exit $?
WELLFLOW_PERSISTENT_BWD=0 timeout -k 10 300 python bench.py || exit $?
timeout -k 10 300 python bench.py || exit $?
