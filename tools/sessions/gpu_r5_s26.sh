# persistent run-ahead: phase stamps of the last step and the grid barrier
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s26 || exit 1
timeout -k 10 120 python tools/stamp_pst.py --steps 20 > gpurun_out/r5s26/stamps20.log 2>&1; rc=$?; cat gpurun_out/r5s26/stamps20.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python tools/stamp_pst.py --steps 200 --reps 3 > gpurun_out/r5s26/stamps200.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r5s26/stamps200.log; [ $rc -eq 0 ] || exit 1
