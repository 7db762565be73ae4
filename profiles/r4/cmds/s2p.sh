# round 4, session 2b: kernel traces (per-kernel stats) of the CNN, LSTM and MLP benches
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_cnn -o run \
  -- python3 bench.py --model cnn --steps 50 --warmup 5 > gpurun_out/r4/prof_cnn.log 2>&1 || { tail -30 gpurun_out/r4/prof_cnn.log; exit 1; }
find gpurun_out/r4/prof_cnn -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_lstm -o run \
  -- python3 bench.py --secondary none --parity none > gpurun_out/r4/prof_lstm.log 2>&1 || { tail -30 gpurun_out/r4/prof_lstm.log; exit 1; }
find gpurun_out/r4/prof_lstm -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/prof_mlp -o run \
  -- python3 bench.py --model mlp --steps 50 --warmup 5 > gpurun_out/r4/prof_mlp.log 2>&1 || { tail -30 gpurun_out/r4/prof_mlp.log; exit 1; }
find gpurun_out/r4/prof_mlp -name "*kernel_stats.csv" -exec python3 tools/kstats.py {} \;
