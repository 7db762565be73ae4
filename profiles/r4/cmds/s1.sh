# round 4, session 1: the fused CNN kernels (tests, then a kernel trace of the CNN bench), the
# production-build diag-switch test, the sync-buffer-offset graph test, the parity test, then
# bench.py (headline + secondaries + parity). Every GPU step has its own limit; && chains them.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_engines_gpu.py -k "cnn" \
  > gpurun_out/r4/s1_cnn_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r4/s1_cnn_tests.log; [ $rc -eq 0 ] || { tail -80 gpurun_out/r4/s1_cnn_tests.log; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_cnn_fused -o run \
  -- python3 bench.py --model cnn --steps 50 --warmup 5 > gpurun_out/r4/prof_cnn_fused.log 2>&1 || { tail -30 gpurun_out/r4/prof_cnn_fused.log; exit 1; }
grep '^{' gpurun_out/r4/prof_cnn_fused.log
find gpurun_out/r4/prof_cnn_fused -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \;
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_step_gpu.py::test_cnn_dropout_mask_differs_per_replay \
  tests/test_kernels_gpu.py::test_diag_env_ignored_by_production_build \
  tests/test_kernels_gpu.py::test_persistent_sync_buffer_at_offset_under_graph_replay \
  tests/test_numerics_gpu.py::test_lstm_headline_adam_trajectory_within_2pct \
  > gpurun_out/r4/s1_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r4/s1_tests.log; [ $rc -eq 0 ] || { tail -60 gpurun_out/r4/s1_tests.log; exit $rc; }
timeout -k 10 400 python bench.py > gpurun_out/r4/s1_bench.log 2>&1 || { tail -20 gpurun_out/r4/s1_bench.log; exit 1; }
grep '^{' gpurun_out/r4/s1_bench.log
