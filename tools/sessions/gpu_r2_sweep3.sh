#!/bin/bash
# R (64-deep sub-tiles per LDS ring slot) sweep: GEMM tests at R 1 / forced 2 and 4, then shapes at cfg 10/11/13 x R 1/2/4
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/sw3
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k gemm --timeout 120 --timeout-method thread > gpurun_out/sw3/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/sw3/pytest.log; [ $rc -ne 0 ] && exit $rc
JDT_GEMM_R=4 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k gemm --timeout 120 --timeout-method thread > gpurun_out/sw3/pytest_r4.log 2>&1
rc=$?; echo "tests r4 rc=$rc"; tail -2 gpurun_out/sw3/pytest_r4.log; [ $rc -ne 0 ] && exit $rc
for c in 10 11 13; do for r in 1 2 4; do
  timeout -k 10 150 python tools/bench_gemm.py --cfg $c --r $r --json gpurun_out/sw3/cfg${c}_r$r.json > gpurun_out/sw3/cfg${c}_r$r.log 2>&1 || { echo "cfg $c r $r rc=$?"; tail -3 gpurun_out/sw3/cfg${c}_r$r.log; exit 1; }
done; echo "cfg $c done"; done
