cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s35 || exit 1
timeout -k 10 120 python tools/stamp_deep.py > gpurun_out/r5s35/deep.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r5s35/deep.log | tail -45; [ $rc -eq 0 ] || exit 1
