#!/bin/bash
# LN with DPP reductions + preloaded affine params: tests, sweep, transformer bench
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/ln2
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_transformer.py -q -x -k "layernorm or ln or transformer or lm" --timeout 120 --timeout-method thread > gpurun_out/ln2/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/ln2/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/bench_ln.py > gpurun_out/ln2/ln.log 2>&1 || exit $?; grep -v amdgpu gpurun_out/ln2/ln.log
for mode in "--merge-microbatches" ""; do
  timeout -k 10 200 python bench.py --strategy pp --model transformer $mode --steps 300 --warmup 30 > gpurun_out/ln2/b.log 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/ln2/b.log; exit 1; }
  echo "mode='$mode': $(grep '^{' gpurun_out/ln2/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
done
