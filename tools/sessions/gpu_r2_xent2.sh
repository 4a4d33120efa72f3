#!/bin/bash
# grid_sum column sums / metrics in the softmax-CE: tests, A/B timing, transformer + DP fused bench
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/xe3
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_reference_loss_fn.py -q -x -k "xent or softmax or transformer or lm or dp or reference or pipeline" --timeout 120 --timeout-method thread > gpurun_out/xe3/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/xe3/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/bench_xent.py > gpurun_out/xe3/x.log 2>&1 || exit $?; grep -v amdgpu gpurun_out/xe3/x.log
for a in "--strategy pp --model transformer --merge-microbatches" "--strategy pp --model transformer" "--accum fused"; do
  timeout -k 10 200 python bench.py $a --steps 300 --warmup 30 > gpurun_out/xe3/b.log 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/xe3/b.log; exit 1; }
  echo "'$a': $(grep '^{' gpurun_out/xe3/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
done
