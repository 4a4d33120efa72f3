#!/bin/bash
# transformer loop / merged with the revised table + epilogue rule, then GEMM tests
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/abf
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/abf/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/abf/pytest.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for mode in "" "--merge-microbatches"; do
  timeout -k 10 200 python bench.py --strategy pp --model transformer $mode --steps 300 --warmup 30 > gpurun_out/abf/b.log 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/abf/b.log; exit 1; }
  echo "mode='$mode': $(grep '^{' gpurun_out/abf/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
done
done
