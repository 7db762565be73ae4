# round 4, session 3: submitted-job throughput at the DEFAULT batch (mean over epochs >= 2)
# for the three job models, then a kernel + copy trace of one online job (per-chunk timeline).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
for m in mlp mlp_online lstm; do
  timeout -k 10 400 python -u tools/job_throughput.py --model $m --default-batch --epochs 6 \
    --out gpurun_out/r4/job_${m}_default.json > gpurun_out/r4/job_${m}_default.log 2>&1 || { tail -30 gpurun_out/r4/job_${m}_default.log; exit 1; }
  tail -3 gpurun_out/r4/job_${m}_default.log | cut -c1-600
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r4/trace_online -o run \
  -- python3 tools/job_throughput.py --model mlp_online --default-batch --epochs 4 > gpurun_out/r4/trace_online.log 2>&1 || { tail -30 gpurun_out/r4/trace_online.log; exit 1; }
K=$(find gpurun_out/r4/trace_online -name "*kernel_trace.csv" | head -1)
C=$(find gpurun_out/r4/trace_online -name "*memory_copy_trace.csv" | head -1)
python3 tools/chunk_timeline.py "$K" "$C" --marker mlp2_step --json gpurun_out/r4/online_chunks.json | cut -c1-300
rm -f "$K" "$C"
