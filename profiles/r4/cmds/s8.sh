# round 4, session 8: online job per-chunk rates (device-timed) + paired parity
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u tools/job_throughput.py --model mlp_online --default-batch --epochs 6 \
  --out gpurun_out/r4/job_mlp_online_default_dev.json > gpurun_out/r4/job_mlp_online_default_dev.log 2>&1 || { tail -30 gpurun_out/r4/job_mlp_online_default_dev.log; exit 1; }
tail -1 gpurun_out/r4/job_mlp_online_default_dev.log | cut -c1-900
bash profiles/r4/cmds/s4.sh
