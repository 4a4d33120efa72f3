#!/bin/bash
# Round 4 session 2: FSDP collective phase stamps (N = 2 / 4 sharing the GPU), the
# 4-layer FSDP8 timeout with per-phase diagnostics, multi-stage pipeline microbatch
# streams A/B (JDT_MB_STREAMS=1 vs default) at N = 4 / 8, pipeline GPU tests.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s2
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py -x -v -k "pipeline or transformer" --timeout 240 \
  --timeout-method thread > gpurun_out/s2/pytest_pp.log 2>&1
rc=$?; echo "pytest pipeline (streams) rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/s2/pytest_pp.log | tail -12
[ $rc -ne 0 ] && { tail -40 gpurun_out/s2/pytest_pp.log; exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_grad_scale_gpu.py -x -v -k pipeline --timeout 240 \
  --timeout-method thread > gpurun_out/s2/pytest_ppscale.log 2>&1
rc=$?; echo "pytest pipeline grad scale rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/s2/pytest_ppscale.log | tail -6
[ $rc -ne 0 ] && { tail -40 gpurun_out/s2/pytest_ppscale.log; exit $rc; }
for cfg in "2 2" "2 4" "4 2"; do
  set -- $cfg
  timeout -k 10 180 python tools/stamp_xg_fsdp.py --ranks $1 --layers $2 > gpurun_out/s2/stamp_r$1_l$2.log 2>&1; rc=$?
  echo "== stamps ranks $1 layers $2 rc=$rc"; grep -v "amdgpu.ids\|socket.cpp\|Gloo" gpurun_out/s2/stamp_r$1_l$2.log | tail -9
  fatal $rc && exit $rc
done
export JDT_BACKEND=gloo
: > gpurun_out/s2/bench.jsonl
i=0
run() {  # n, env, args
  i=$((i+1))
  env $2 timeout -k 10 240 python bench.py --gpus $1 --steps 100 --warmup 10 $3 > gpurun_out/s2/b$i.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "N=$1 [$2] '$3' rc=$rc"; grep -v "^\[rank[1-9]" gpurun_out/s2/b$i.log | grep -iE "error|timed|Traceback" | tail -6; fatal $rc && exit $rc; return 0; }
  echo "== N=$1 [$2] $3: $(grep '^{' gpurun_out/s2/b$i.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["config"].get("stage_streams"), j["config"].get("num_microbatches"))')"
  grep '^{' gpurun_out/s2/b$i.log >> gpurun_out/s2/bench.jsonl
}
run 8 "JDT_X=0" "--strategy fsdp --num-layers 4"
run 8 "GPU_MAX_HW_QUEUES=2" "--strategy fsdp --num-layers 4"
for rep in 1 2; do
  for st in 1 4; do
    run 4 "JDT_MB_STREAMS=$st" "--strategy pp --hidden-layers 8"
    run 4 "JDT_MB_STREAMS=$st" "--strategy pp --hidden-layers 8 --microbatches 4"
    run 4 "JDT_MB_STREAMS=$st" "--strategy pp --dp 2 --model transformer"
    run 4 "JDT_MB_STREAMS=$st" "--strategy pp --dp 2 --model transformer --microbatches 4"
  done
done
run 2 "JDT_X=0" "--strategy fsdp"
run 2 "JDT_X=0" ""
run 8 "JDT_X=0" "--strategy pp --hidden-layers 8"
run 8 "JDT_X=0" "--strategy pp --dp 2 --model transformer"
run 8 "JDT_X=0" "--strategy pp --dp 2 --model transformer --microbatches 4"
echo done
