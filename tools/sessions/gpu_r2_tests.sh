#!/bin/bash
# GPU test tiers: new scale-sensitive tests + xGMI tests first, then the whole GPU suite, then benches.
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_grad_scale_gpu.py tests/test_xgmi_gpu.py -v --timeout 200 --timeout-method thread > gpurun_out/pytest_scale_xgmi.log 2>&1
rc=$?; echo "scale+xgmi rc=$rc"; tail -4 gpurun_out/pytest_scale_xgmi.log
fatal $rc && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "all-gpu rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
fatal $rc && exit $rc
JDT_BACKEND=gloo timeout -k 10 200 python bench.py --gpus 2 --steps 200 --warmup 20 > gpurun_out/bench2_gloo.log 2>&1
rc=$?; echo "bench2 rc=$rc"; grep -v Gloo gpurun_out/bench2_gloo.log | tail -3
fatal $rc && exit $rc
JDT_BACKEND=gloo timeout -k 10 200 python bench.py --gpus 4 --steps 200 --warmup 20 > gpurun_out/bench4_gloo.log 2>&1
rc=$?; echo "bench4 rc=$rc"; grep -v Gloo gpurun_out/bench4_gloo.log | tail -3
exit $rc
