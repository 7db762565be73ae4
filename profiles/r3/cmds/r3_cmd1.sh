set -o pipefail
bash tools/gpu.sh tests; rc=$?; echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench1.log 2>&1; rc=$?; tail -2 gpurun_out/bench1.log; echo "bench rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/pin_job.sh; echo "pin rc=$?"
