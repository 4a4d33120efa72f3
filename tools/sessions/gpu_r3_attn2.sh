#!/bin/bash
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/attn
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attn128 or flash_attention or attention_fwd_bwd" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/attn/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/bench_attn.py > gpurun_out/attn/bench_attn.log 2>&1 || exit $?
cat gpurun_out/attn/bench_attn.log
