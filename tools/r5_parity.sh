# round-5 fixed-epoch paired LSTM val-MSE parity: both precisions run
# exactly EPOCHS epochs (patience above the cap: no early-stopping noise), best val MSE paired
# per seed; SEEDS split over GPU calls and pooled with tools/parity.py --merge.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 ${TL:-1080} python -u tools/parity.py --model lstm --batch 0 --epochs ${EPOCHS:-40} --patience 1000 \
  --seeds $SEEDS --out gpurun_out/r5/parity_lstm_fixed_$TAG.json > gpurun_out/r5/parity_lstm_fixed_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/r5/parity_lstm_fixed_$TAG.log | cut -c1-600
exit $rc
