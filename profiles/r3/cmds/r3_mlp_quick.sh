set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_engines_gpu.py -k "mlp" > gpurun_out/tm.log 2>&1; rc=$?; tail -2 gpurun_out/tm.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/tm.log; exit $rc; }
BATCHES="16384 262144" bash tools/r3_mlp_scan.sh
