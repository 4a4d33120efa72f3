#!/bin/bash
# Round-2 GPU check: GPU tests, 1-GPU bench, 2-rank shared-GPU bench (gloo process group, xGMI kernels).
# Stops at the first GPU fault / abort / timeout (exit codes 124, 134, 137, 139).
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
fatal $rc && exit $rc
timeout -k 10 150 python bench.py > gpurun_out/bench1.log 2>&1
rc=$?; echo "bench1 rc=$rc"; tail -1 gpurun_out/bench1.log
fatal $rc && exit $rc
JDT_BACKEND=gloo timeout -k 10 200 python bench.py --gpus 2 --steps 200 --warmup 20 > gpurun_out/bench2_gloo.log 2>&1
rc=$?; echo "bench2 rc=$rc"; tail -1 gpurun_out/bench2_gloo.log
exit $rc
