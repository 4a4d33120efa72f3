#!/bin/bash
# deep LDS ring sweep: GEMM tests, then every shape at cfg 10/11/13 with deep 0/1, auto, ksweep
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/sw2
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k gemm --timeout 120 --timeout-method thread > gpurun_out/sw2/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/sw2/pytest.log; [ $rc -ne 0 ] && exit $rc
for c in 10 11 13; do for d in 0 1; do
  timeout -k 10 150 python tools/bench_gemm.py --cfg $c --deep $d --json gpurun_out/sw2/cfg${c}_d$d.json > gpurun_out/sw2/cfg${c}_d$d.log 2>&1 || { echo "cfg $c d $d rc=$?"; tail -3 gpurun_out/sw2/cfg${c}_d$d.log; exit 1; }
done; echo "cfg $c done"; done
timeout -k 10 150 python tools/bench_gemm.py --json gpurun_out/sw2/auto.json > gpurun_out/sw2/auto.log 2>&1; echo "auto rc=$?"
