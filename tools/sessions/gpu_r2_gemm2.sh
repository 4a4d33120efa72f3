#!/bin/bash
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1
rc=$?; echo "gemm tests rc=$rc"; tail -5 gpurun_out/pytest_gemm.log; case $rc in 124|134|137|139) exit $rc;; esac
for c in -1 14; do echo "=== cfg $c"; timeout -k 10 120 python tools/bench_gemm.py --cfg $c --json gpurun_out/gemm2_cfg$c.json || exit $?; done
echo "=== groups"; timeout -k 10 120 python tools/bench_gemm.py --only none --groups 64,128,0 --json gpurun_out/gemm2_groups.json || exit $?
