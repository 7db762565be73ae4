#!/bin/bash
# round-5 closing GPU pass: job-vs-bench for the three job configs, the MLP PMC table, and the
# default bench line (headline + secondaries + parity). Output under gpurun_out/r5/final2.
set -o pipefail
O=gpurun_out/r5/final2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/job_throughput.py --model mlp --epochs 6 --out $O/job_mlp.json > $O/job_mlp.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/job_throughput.py --model mlp_online --epochs 12 --out $O/job_mlp_online.json > $O/job_mlp_online.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/job_throughput.py --model lstm --epochs 4 --out $O/job_lstm.json > $O/job_lstm.log 2>&1 || exit 1
bash tools/pmc4.sh $O/pmc_mlp mlp "step128 dw2g mlp2" > $O/pmc.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || exit 1
echo done
