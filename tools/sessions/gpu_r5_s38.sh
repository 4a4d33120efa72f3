#!/bin/bash
# The md_bwd AdamW pin kept out of the exchange (TX) variants: the DP / FSDP over xGMI tests (one-launch
# deep DP at 2 ranks again), the deep / pipeline tests, and the 4-layer bench (pin gain retained).
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s38
timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py tests/test_kernels_gpu.py tests/test_pp_chain_gpu.py tests/test_grad_scale_gpu.py -m gpu -q -rs --timeout 300 --timeout-method thread \
  > gpurun_out/r5s38/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r5s38/pytest.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r5s38/pytest.log | head -20; exit $rc; }
for r in 1 2; do
  timeout -k 10 180 python bench.py --steps 300 --warmup 30 --num-layers 4 > gpurun_out/r5s38/b4_$r.log 2>&1 || { tail -5 gpurun_out/r5s38/b4_$r.log; exit 1; }
  grep '^{' gpurun_out/r5s38/b4_$r.log | cut -c1-120
done
echo done
