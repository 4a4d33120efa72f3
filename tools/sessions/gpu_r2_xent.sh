#!/bin/bash
# DPP reductions in the wide softmax-CE: tests + rows-per-wave sweep
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/xe
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "xent or softmax or transformer or lm or ln" --timeout 120 --timeout-method thread > gpurun_out/xe/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/xe/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/bench_xent.py > gpurun_out/xe/x.log 2>&1 || exit $?; grep -v amdgpu gpurun_out/xe/x.log
