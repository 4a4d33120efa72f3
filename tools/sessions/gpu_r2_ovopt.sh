#!/bin/bash
# Overlapped (layer-by-layer, side-stream) AdamW on the 1-GPU transformer step: bitwise test, A/B bench
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/ovopt
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "overlapped_adamw or single_stage or transformer_step" -s > gpurun_out/ovopt/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/ovopt/pytest.log | tail -8; [ $rc -ne 0 ] && exit $rc
val() { grep '^{' "$1" | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["details"]["final_loss"])'; }
for rep in 1 2; do
  for ov in 0 1; do
    JDT_OVERLAP_OPT=$ov timeout -k 10 180 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > gpurun_out/ovopt/b.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { tail -5 gpurun_out/ovopt/b.log; exit $rc; }
    echo "rep $rep overlap=$ov: $(val gpurun_out/ovopt/b.log)"
  done
done
