#!/bin/bash
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/gelu
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_transformer.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gelu/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/gelu/pytest.log; [ $rc -ne 0 ] && exit $rc
for a in "--strategy pp --model transformer" "--strategy pp --model transformer --microbatch-passes"; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 $a > gpurun_out/gelu/b.log 2>&1 || exit 1
  echo "'$a': $(grep '^{' gpurun_out/gelu/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
done
timeout -k 10 200 python tools/bench_ln_gemm.py 2>&1 | grep -v amdgpu.ids
