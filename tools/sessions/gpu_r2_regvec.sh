#!/bin/bash
# vectorised epilogue in the register-staged GEMM: GEMM tests, shapes, generic-path benches (vec on / off)
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/rv
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/rv/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/rv/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python tools/bench_gemm.py --only "mlp fwd,mlp dW,fc2 dW,fc1 dW" > gpurun_out/rv/g.log 2>&1 || exit $?; grep -v amdgpu gpurun_out/rv/g.log
for rep in 1 2; do for e in 1 0; do for a in "--accum loop" "--accum fused" "--strategy pp --model transformer"; do
  JDT_GEMM_EPI_VEC=$e timeout -k 10 200 python bench.py $a --steps 300 --warmup 30 > gpurun_out/rv/b.log 2>&1 || { echo "rc=$?"; exit 1; }
  echo "rep $rep vec=$e '$a': $(grep '^{' gpurun_out/rv/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
done; done; done
