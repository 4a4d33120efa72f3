#!/bin/bash
# One-stage GPipe (8 hidden layers, deep engine) with the layer-0 run-ahead: tests, A/B bench
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/ppa
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_stage_gpu.py \
  -k "pipeline_single_stage_run_ahead or deep_run_ahead or single_stage or fused_stage" > gpurun_out/ppa/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/ppa/pytest.log | tail -10; [ $rc -ne 0 ] && exit $rc
val() { grep '^{' "$1" | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["details"]["final_loss"])'; }
for rep in 1 2; do
  for ah in 0 1; do
    JDT_MLP2_AHEAD=$ah timeout -k 10 120 python bench.py --strategy pp --hidden-layers 8 --steps 300 --warmup 30 > gpurun_out/ppa/b.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { tail -5 gpurun_out/ppa/b.log; exit $rc; }
    echo "rep $rep ahead=$ah pp8: $(val gpurun_out/ppa/b.log)"
  done
done
