#!/bin/bash
# DP minibatch loop on the fused per-layer kernels: all GPU tests touching DP / fused stage / xGMI, then benches
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/fl
timeout -k 10 600 python -u -m pytest tests/test_fused_stage_gpu.py tests/test_grad_scale_gpu.py tests/test_kernels_gpu.py tests/test_deterministic_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/fl/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/fl/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u -m pytest tests/test_xgmi_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/fl/pytest_xg.log 2>&1
rc=$?; echo "xgmi tests rc=$rc"; tail -3 gpurun_out/fl/pytest_xg.log; [ $rc -ne 0 ] && exit $rc
for a in "--accum loop" "--accum loop --num-layers 4" "--accum scan"; do for fl in 1 0; do
  JDT_FUSED_LOOP=$fl timeout -k 10 200 python bench.py $a --steps 300 --warmup 30 > gpurun_out/fl/b.log 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/fl/b.log; exit 1; }
  echo "fused_loop=$fl '$a': $(grep '^{' gpurun_out/fl/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
done; done
