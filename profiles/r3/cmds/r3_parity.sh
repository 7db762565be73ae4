#!/bin/bash
# paired converged val-MSE parity, seeds given by SEEDS (one GPU call per group of seeds)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${TLIM:-1100} python -u tools/parity.py --model ${MODEL:-lstm} --seeds ${SEEDS:-0} \
  --out gpurun_out/parity_${MODEL:-lstm}_${TAG:-s0}.json > gpurun_out/parity_${MODEL:-lstm}_${TAG:-s0}.log 2>&1
rc=$?; tail -12 gpurun_out/parity_${MODEL:-lstm}_${TAG:-s0}.log | cut -c1-400; exit $rc
