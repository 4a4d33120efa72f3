#!/bin/bash
# FSDP fused-loop gradient-scale diagnostic, the GEMM main-loop lab, then the rest of the GPU suite (no -x)
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/d1
timeout -k 10 300 python -u tools/diag_fsdp_loop.py > gpurun_out/d1/diag.log 2>&1; rc=$?
echo "diag rc=$rc"; grep "^ws=" gpurun_out/d1/diag.log; tail -3 gpurun_out/d1/diag.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 200 ./tools/gemm_lab/gemm_lab > gpurun_out/d1/lab.log 2>&1; rc=$?
echo "lab rc=$rc"; cat gpurun_out/d1/lab.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "not fsdp_loop_sgd" > gpurun_out/d1/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/d1/pytest.log | tail -20
