set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5diag
export TMPDIR=/tmp
PB_ROUNDS=3 timeout -k 10 300 python -u tools/pb_time.py 0,1,2,4,8,16,128,4096 > gpurun_out/r5diag/pb_time.txt 2>&1 && \
timeout -k 10 200 python -u tools/pf_timeline.py 16 > gpurun_out/r5diag/pf_timeline.txt 2>&1 && \
timeout -k 10 200 python -u tools/pf_time.py 0,1,2,4,8 > gpurun_out/r5diag/pf_time.txt 2>&1
echo rc=$?
