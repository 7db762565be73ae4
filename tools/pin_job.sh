#!/bin/bash
# The round-2 open failure, with the round-3 completion STAT block: the LSTM job with pinned
# evaluation slots (WELLFLOW_EVAL_PIN=1) between graph-replayed epochs. check_device_errors
# raises with the first-exit record (block, step, reason, words seen); exit status 1 is that
# expected Python error, anything else (GPU fault, abort, time limit) ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
WELLFLOW_EVAL_PIN=${PIN:-1} timeout -k 10 400 python -u tools/job_throughput.py --model lstm --epochs ${EPOCHS:-3} \
  > gpurun_out/pin_job.log 2>&1; rc=$?
tail -5 gpurun_out/pin_job.log
exit $rc
