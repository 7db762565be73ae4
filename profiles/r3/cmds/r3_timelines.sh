export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/pf_timeline.py 16 > gpurun_out/pf_timeline.log 2>&1; echo "pf rc=$?"; cat gpurun_out/pf_timeline.log | grep -v amdgpu.ids
timeout -k 10 200 python tools/pb_timeline.py 32 > gpurun_out/pb_timeline.log 2>&1; echo "pb rc=$?"; cat gpurun_out/pb_timeline.log | grep -v amdgpu.ids
