#!/bin/bash
# 8-wave LDS-DMA GEMM tiles: numerics vs the 4-wave tile, K sweep, transformer shapes
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/w8
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "8wave or vec_epilogue" > gpurun_out/w8/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/w8/pytest.log; exit 1; }
tail -2 gpurun_out/w8/pytest.log
timeout -k 10 300 python tools/gemm_ksweep.py --cfgs 12,14,15,16,17,18 > gpurun_out/w8/ksweep.log 2>&1 || { echo "ksweep rc=$?"; tail -5 gpurun_out/w8/ksweep.log; exit 1; }
grep -v amdgpu.ids gpurun_out/w8/ksweep.log
for c in -1 15 16 17 18; do
  timeout -k 10 200 python tools/bench_gemm.py --cfg $c > gpurun_out/w8/bg.log 2>&1 || { echo "bench_gemm rc=$?"; tail -5 gpurun_out/w8/bg.log; exit 1; }
  echo "== cfg $c"; grep -v amdgpu.ids gpurun_out/w8/bg.log | grep -v "^group\|grouped"
done
