cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s30 || exit 1
timeout -k 10 120 python tools/probe_pst_launch.py > gpurun_out/r5s30/probe.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r5s30/probe.log | tail -4; [ $rc -eq 0 ] || exit 1
