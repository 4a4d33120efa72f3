#!/bin/bash
# vectorised GEMM epilogue: GEMM/transformer numerics tests, K sweep (old vs new epilogue), shape table, transformer bench
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/epi
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_transformer.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/epi/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/epi/pytest.log; fatal $rc && exit $rc; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/gemm_ksweep.py --epi 0,1 --layouts mk/kn,km/kn > gpurun_out/epi/ksweep.log 2>&1 || exit $?
timeout -k 10 150 python tools/bench_gemm.py --json gpurun_out/epi/gemm.json > gpurun_out/epi/gemm.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --strategy pp --model transformer --merge-microbatches --steps 200 --warmup 20 > gpurun_out/epi/tf.log 2>&1; rc=$?
echo "tf rc=$rc"; grep '^{' gpurun_out/epi/tf.log | cut -c1-250
