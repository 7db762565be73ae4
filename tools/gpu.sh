#!/bin/bash
# One entry point for every GPU-box run (replaces the round-1 one-off gpu_*.sh scripts).
#   tools/gpu.sh tests            GPU test tier (+ smoke)
#   tools/gpu.sh bench [args]     bench.py for lstm, mlp, mlp_online (extra args passed through)
#   tools/gpu.sh prof TAG [args]  rocprofv3 kernel-trace --stats of bench.py -> gpurun_out/prof_TAG
#   tools/gpu.sh pmc TAG "CTRS" [args]  one rocprofv3 --pmc pass (<= 8 SQ counters) -> gpurun_out/pmc_TAG
#   tools/gpu.sh all              tests + smoke + the three benches
#   tools/gpu.sh sweep VAR "v1 v2 .." [bench args]   bench.py once per env value VAR=v (e.g.
#                                 WELLFLOW_MLP_STEP128, WELLFLOW_DW_SLAB)
#   tools/gpu.sh ksweep VAR "v1 v2 .." KERNEL [bench args]  the same under rocprofv3 --kernel-trace,
#                                 printing the stats line of kernels matching KERNEL per value
#   tools/gpu.sh pmcsets "SET1" "SET2" ..   one rocprofv3 --pmc pass per counter set over a 2-step
#                                 LSTM bench (--no-graph; PMC_ARGS overrides the bench args)
#                                 -> gpurun_out/pmc/setN (tools/pmc_table.py summarises them)
#   tools/gpu.sh tool SCRIPT [args]   a diagnostic script under tools/ (pf_time.py, pb_time.py,
#                                 pf_timeline.py, pb_timeline.py, tune_lstm.py, dw_vs_blas.py, ...)
# Every GPU step has its own time limit and the steps are chained: the first failure ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
what="$1"; shift || true

run_tests() {
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/tgpu.log 2>&1; local rc=$?
  grep -E "passed|failed|error" gpurun_out/tgpu.log | tail -3
  if [ $rc -ne 0 ]; then tail -60 gpurun_out/tgpu.log; return $rc; fi
  timeout -k 10 300 python __graft_entry__.py smoke
}

run_bench() {
  timeout -k 10 300 python bench.py "$@" || return $?
  timeout -k 10 300 python bench.py --model mlp "$@" || return $?
  timeout -k 10 300 python bench.py --model mlp_online "$@"
}

case "$what" in
  tests) run_tests ;;
  bench) run_bench "$@" ;;
  all) run_tests && run_bench "$@" ;;
  prof)
    tag="$1"; shift
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/prof_$tag" -o run \
      -- python3 bench.py "$@" > "gpurun_out/prof_$tag.log" 2>&1; rc=$?
    tail -3 "gpurun_out/prof_$tag.log"
    find "gpurun_out/prof_$tag" -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \;
    exit $rc ;;
  pmc)
    tag="$1"; ctrs="$2"; shift 2
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d "gpurun_out/pmc_$tag" -o run \
      -- python3 bench.py "$@" > "gpurun_out/pmc_$tag.log" 2>&1; rc=$?
    tail -3 "gpurun_out/pmc_$tag.log"
    exit $rc ;;
  sweep)
    var="$1"; vals="$2"; shift 2
    for v in $vals; do
      echo "== $var=$v"
      env "$var=$v" timeout -k 10 200 python bench.py "$@" || exit $?
    done ;;
  ksweep)
    var="$1"; vals="$2"; kern="$3"; shift 3
    for v in $vals; do
      env "$var=$v" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/ks_$v" -o run \
        -- python3 bench.py "$@" > "gpurun_out/ks_$v.log" 2>&1 || exit $?
      echo "$var=$v $(python3 tools/kstats.py "gpurun_out/ks_$v/run_kernel_stats.csv" | grep "$kern")"
    done ;;
  pmcsets)
    rm -rf gpurun_out/pmc
    mkdir -p gpurun_out/pmc
    i=0
    for set in "$@"; do
      i=$((i+1))
      timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/set$i -o run \
        -- python3 bench.py ${PMC_ARGS:---steps 2 --warmup 1 --no-graph} > gpurun_out/pmc/set$i.log 2>&1 || { tail -5 gpurun_out/pmc/set$i.log; exit 1; }
    done ;;
  tool)
    script="$1"; shift
    timeout -k 10 600 python "tools/$script" "$@" ;;
  *) echo "usage: tools/gpu.sh tests|bench|all|prof TAG|pmc TAG CTRS|sweep|ksweep|pmcsets|tool [args]"; exit 2 ;;
esac
