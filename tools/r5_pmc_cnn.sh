# CNN PMC before (round-4 tree, r4tree/) and after (this tree): tools/pmc4.sh in each
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5/pmc_cnn_after gpurun_out/r5/pmc_cnn_before
bash tools/pmc4.sh gpurun_out/r5/pmc_cnn_after cnn "cnn_fwd cnn_bwd" > gpurun_out/r5/pmc_cnn_after/run.log 2>&1 || { tail -5 gpurun_out/r5/pmc_cnn_after/run.log; exit 1; }
cat gpurun_out/r5/pmc_cnn_after/pmc_table.md
R=$GRAFT_REPO_ROOT; GRAFT_REPO_ROOT=$R/r4tree bash $R/tools/pmc4.sh $R/gpurun_out/r5/pmc_cnn_before cnn "cnn_fwd cnn_bwd" > $R/gpurun_out/r5/pmc_cnn_before/run.log 2>&1 || { tail -5 $R/gpurun_out/r5/pmc_cnn_before/run.log; exit 1; }
cat $R/gpurun_out/r5/pmc_cnn_before/pmc_table.md
