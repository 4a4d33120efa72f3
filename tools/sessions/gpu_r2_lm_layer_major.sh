#!/bin/bash
# transformer single stage layer-major by default (dropout-free): tests + benches
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/lm
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_stage_gpu.py -q -x -k "pipeline or stage or transformer or lm" --timeout 200 --timeout-method thread > gpurun_out/lm/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/lm/pytest.log; [ $rc -ne 0 ] && exit $rc
for a in "--strategy pp --model transformer" "--strategy pp --hidden-layers 8"; do
  timeout -k 10 200 python bench.py $a --steps 300 --warmup 30 > gpurun_out/lm/b.log 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/lm/b.log; exit 1; }
  echo "'$a': $(grep '^{' gpurun_out/lm/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["config"].get("single_stage_mode"))')"
done
