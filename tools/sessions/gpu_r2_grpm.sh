#!/bin/bash
# GEMM tile row-group order (JDT_GEMM_GROUP_M) x tile config: K sweep + transformer shapes
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/gm
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "8wave" > gpurun_out/gm/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/gm/pytest.log; exit 1; }
tail -1 gpurun_out/gm/pytest.log
timeout -k 10 300 python tools/gemm_ksweep.py --cfgs 11,12,15 --group-m 0,2,4,8 --ks 512,2048 > gpurun_out/gm/ksweep.log 2>&1 || { echo "ksweep rc=$?"; tail -5 gpurun_out/gm/ksweep.log; exit 1; }
grep -v amdgpu.ids gpurun_out/gm/ksweep.log
for spec in "-1:0" "-1:4" "-1:8" "15:4" "15:8" "10:4" "10:8"; do
  c=${spec%%:*}; gm=${spec#*:}
  JDT_GEMM_GROUP_M=$gm timeout -k 10 200 python tools/bench_gemm.py --cfg $c > gpurun_out/gm/bg.log 2>&1 || { echo "bench_gemm rc=$?"; tail -5 gpurun_out/gm/bg.log; exit 1; }
  echo "== cfg $c group_m $gm"; grep -v amdgpu.ids gpurun_out/gm/bg.log | grep " 2k\|hyb\|^shape"
done
