set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_numerics_gpu.py tests/test_job_gpu.py > gpurun_out/t7.log 2>&1; rc=$?
tail -3 gpurun_out/t7.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/t7.log | head -30; exit $rc; }
timeout -k 10 400 python -u tools/job_throughput.py --model lstm --default-batch --out gpurun_out/job_default.json > gpurun_out/job_default.log 2>&1 || { tail -20 gpurun_out/job_default.log; exit 1; }
tail -1 gpurun_out/job_default.log | cut -c1-600
timeout -k 10 400 python -u tools/job_throughput.py --model lstm --default-batch --wells 90 --out gpurun_out/job_f100.json > gpurun_out/job_f100.log 2>&1 || { tail -20 gpurun_out/job_f100.log; exit 1; }
tail -1 gpurun_out/job_f100.log | cut -c1-600
