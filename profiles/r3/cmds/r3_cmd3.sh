set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu.sh tests; rc=$?; echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench3.log 2>&1; rc=$?; grep "^{" gpurun_out/bench3.log; echo "bench rc=$rc"
