#!/bin/bash
# generic DP minibatch loop after removing the per-minibatch device int ops: tests + bench
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/loop
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_grad_scale_gpu.py tests/test_reference_loss_fn.py -q -x -k "dp or loop or scan or accum or grad or reference" --timeout 120 --timeout-method thread > gpurun_out/loop/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/loop/pytest.log; [ $rc -ne 0 ] && exit $rc
for a in "--accum loop" "--accum scan" "--accum fused"; do
  timeout -k 10 200 python bench.py $a --steps 300 --warmup 30 > gpurun_out/loop/b.log 2>&1 || { echo "rc=$?"; exit 1; }
  echo "'$a': $(grep '^{' gpurun_out/loop/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
done
