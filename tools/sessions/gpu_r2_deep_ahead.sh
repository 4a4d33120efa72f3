#!/bin/bash
# Deep-MLP run-ahead (layer-0 backward + next layer-0 forward): GPU tests, then A/B bench
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/deep
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "deep_run_ahead or fused_mlp_step or run_ahead or fsdp" > gpurun_out/deep/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/deep/pytest.log | tail -12; [ $rc -ne 0 ] && exit $rc
val() { grep '^{' "$1" | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["details"]["final_loss"])'; }
for rep in 1 2; do
  for ah in 0 1; do
    for L in 4 3; do
      JDT_MLP2_AHEAD=$ah timeout -k 10 120 python bench.py --num-layers $L --steps 300 --warmup 30 > gpurun_out/deep/b.log 2>&1; rc=$?
      [ $rc -ne 0 ] && { tail -5 gpurun_out/deep/b.log; exit $rc; }
      echo "rep $rep ahead=$ah layers=$L: $(val gpurun_out/deep/b.log)"
    done
  done
done
JDT_MLP2_AHEAD=1 timeout -k 10 120 python bench.py --strategy fsdp --num-layers 4 --steps 300 --warmup 30 > gpurun_out/deep/b.log 2>&1; rc=$?
[ $rc -ne 0 ] && { tail -5 gpurun_out/deep/b.log; exit $rc; }
echo "fsdp 4-layer ahead: $(val gpurun_out/deep/b.log)"
