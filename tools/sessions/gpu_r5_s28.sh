cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s28 || exit 1
timeout -k 10 120 python tools/stamp_pst.py --steps 200 --reps 3 > gpurun_out/r5s28/stamps.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r5s28/stamps.log | grep -v "dispatch XCD"; [ $rc -eq 0 ] || exit 1
