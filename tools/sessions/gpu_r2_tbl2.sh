#!/bin/bash
# tune table with 8-wave tiles + tile order: GEMM / transformer tests, shape table, in-model A/B
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/tb2
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_transformer.py > gpurun_out/tb2/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/tb2/pytest.log; exit 1; }
tail -1 gpurun_out/tb2/pytest.log
timeout -k 10 200 python tools/bench_gemm.py --groups 0 --json gpurun_out/tb2/gemm.json > gpurun_out/tb2/bg.log 2>&1 || { echo "bench_gemm rc=$?"; tail -5 gpurun_out/tb2/bg.log; exit 1; }
grep -v amdgpu.ids gpurun_out/tb2/bg.log
for rep in 1 2; do
for gm in 0 -1; do
  for mode in "" "--merge-microbatches"; do
  JDT_GEMM_GROUP_M=$gm timeout -k 10 200 python bench.py --strategy pp --model transformer $mode --steps 300 --warmup 30 > gpurun_out/tb2/b.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/tb2/b.log; exit 1; }
  echo "gm=$gm $mode: $(grep '^{' gpurun_out/tb2/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
  done
done
done
