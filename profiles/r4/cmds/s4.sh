# round 4, session 4: paired converged val-MSE parity at the job's default batch (batch 0 = auto)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
S=${SEEDS:-0,1,2,3,4,5,6,7}; TAG=${TAG:-a}
for M in ${MODELS:-mlp lstm}; do
  timeout -k 10 ${TLIM:-540} python -u tools/parity.py --model $M --seeds $S --batch 0 \
    --out gpurun_out/r4/parity_${M}_${TAG}.json > gpurun_out/r4/parity_${M}_${TAG}.log 2>&1
  rc=$?; tail -6 gpurun_out/r4/parity_${M}_${TAG}.log | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
done
