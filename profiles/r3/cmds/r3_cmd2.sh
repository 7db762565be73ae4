set -o pipefail
# A/B of the round-2 early exit: legacy per-launch memset (4 B past the allocation start,
# WELLFLOW_PF_DBG bit 20) vs the whole-block memset, with pinned eval slots, then legacy unpinned
export TMPDIR=/tmp
mkdir -p gpurun_out
WELLFLOW_PF_DBG=1048576 WELLFLOW_EVAL_PIN=1 timeout -k 10 400 python -u tools/job_throughput.py --model lstm --epochs 3 > gpurun_out/pin_legacy.log 2>&1; rc=$?
echo "legacy+pin rc=$rc"; tail -4 gpurun_out/pin_legacy.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
WELLFLOW_PF_DBG=1048576 WELLFLOW_EVAL_PIN=0 timeout -k 10 400 python -u tools/job_throughput.py --model lstm --epochs 3 > gpurun_out/nopin_legacy.log 2>&1; rc=$?
echo "legacy+nopin rc=$rc"; tail -4 gpurun_out/nopin_legacy.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
WELLFLOW_EVAL_PIN=1 timeout -k 10 400 python -u tools/job_throughput.py --model lstm --epochs 3 > gpurun_out/pin_new.log 2>&1; rc=$?
echo "new+pin rc=$rc"; tail -4 gpurun_out/pin_new.log
