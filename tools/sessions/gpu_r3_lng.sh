#!/bin/bash
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/lng
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "ln_gemm" -x -q --timeout 120 --timeout-method thread > gpurun_out/lng/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/lng/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/bench_ln_gemm.py 2>&1 | grep -v amdgpu.ids
for a in 1 0; do
  JDT_LN_GEMM=$a timeout -k 10 200 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > gpurun_out/lng/b.log 2>&1 || exit 1
  echo "ln_gemm=$a lm: $(grep '^{' gpurun_out/lng/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
done
