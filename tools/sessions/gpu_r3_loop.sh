#!/bin/bash
# DP minibatch loop (reference semantics) on concurrent streams: GPU tests, alternating bench A/B
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/loop
timeout -k 10 300 python -u -m pytest tests/test_grad_scale_gpu.py tests/test_fused_stage_gpu.py -x -q -s --timeout 120 --timeout-method thread -k "generic_gemm or loop_streams or fused_stage" > gpurun_out/loop/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|Error|rel diff" gpurun_out/loop/pytest.log | tail -12
case $rc in 0) ;; *) exit $rc;; esac
for rep in 1 2; do
  for nl in 2 4; do
    for k in 1 2 4; do
      JDT_LOOP_STREAMS=$k timeout -k 10 180 python bench.py --accum loop --num-layers $nl --steps 300 --warmup 20 > gpurun_out/loop/b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/loop/b.log; exit 1; }
      echo "rep $rep layers $nl loop streams $k: $(grep '^{' gpurun_out/loop/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
    done
  done
done
