#!/bin/bash
# whole-head flash backward: attention tests, A/B timing, transformer bench
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/flash
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "attention or transformer or lm" --timeout 120 --timeout-method thread > gpurun_out/flash/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/flash/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/bench_attn.py > gpurun_out/flash/attn.log 2>&1; rc=$?; echo "attn rc=$rc"; grep -v amdgpu gpurun_out/flash/attn.log; fatal $rc && exit $rc
timeout -k 10 200 python bench.py --strategy pp --model transformer --merge-microbatches --steps 300 --warmup 30 > gpurun_out/flash/tf.log 2>&1; rc=$?
echo "tf rc=$rc"; grep '^{' gpurun_out/flash/tf.log | cut -c1-220
