#!/bin/bash
# Fused SGD in the 2-layer engine: tests, then bench A/B (mode 0 + SGD kernel vs fused + run-ahead)
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/sgd
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_grad_scale_gpu.py \
  -k "sgd or run_ahead or fused_mlp_step or loop_kernel" > gpurun_out/sgd/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/sgd/pytest.log | tail -8; [ $rc -ne 0 ] && exit $rc
val() { grep '^{' "$1" | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["details"]["final_loss"], j["config"].get("step_launches"))'; }
for rep in 1 2; do for f in 0 1; do
  JDT_FUSED_SGD=1 JDT_FUSED_OPT=$f timeout -k 10 120 python bench.py --optimizer sgd --steps 300 --warmup 30 > gpurun_out/sgd/b.log 2>&1 || { tail -5 gpurun_out/sgd/b.log; exit 1; }
  echo "rep $rep fused=$f: $(val gpurun_out/sgd/b.log)"
done; done
