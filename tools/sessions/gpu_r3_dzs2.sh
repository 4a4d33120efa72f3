#!/bin/bash
# dZ split on by default: every deep-engine test with it on, the stamps with it on
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/dzs2
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_grad_scale_gpu.py tests/test_fused_stage_gpu.py tests/test_deterministic_gpu.py tests/test_xgmi_gpu.py -q -x --timeout 150 --timeout-method thread -k "dz_split or deep or fused_mode or run_ahead or fused_stage or determin or fsdp or graph_capture or mb_streams or set_batch" > gpurun_out/dzs2/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|Error" gpurun_out/dzs2/pytest.log | tail -8
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 120 python tools/stamp_deep.py --layers 4 > gpurun_out/dzs2/stamp.log 2>&1 || { tail -5 gpurun_out/dzs2/stamp.log; exit 1; }
grep -v amdgpu.ids gpurun_out/dzs2/stamp.log
