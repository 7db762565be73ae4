# kernel trace of the LSTM bench (rocprofv3 --kernel-trace --stats) -> gpurun_out/r5/prof_$1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
tag=$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/prof_$tag -o run \
  -- python3 bench.py --secondary none --parity none "$@" > gpurun_out/r5/prof_$tag.log 2>&1; rc=$?
tail -2 gpurun_out/r5/prof_$tag.log
find gpurun_out/r5/prof_$tag -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \;
exit $rc
