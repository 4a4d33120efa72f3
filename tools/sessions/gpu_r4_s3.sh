#!/bin/bash
# Round 4 session 3: xGMI kernels with batched loads + AdamW prefetch (xg_kernel, one-shot,
# xg_fsdp_kernel): collective tests at 2/4/8 ranks, DP/FSDP equal to one device, grad-scale
# probes, FSDP phase stamps, N = 2 / 4 DP and FSDP rehearsal (A/B against the round-3 rows in
# profiles/r4_eight_rank_rehearsal.txt / r3_closing_run.txt), then the GPU_MAX_HW_QUEUES=2 diagnosis LAST
# (it may end in a native crash, after which nothing else runs).
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s3
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -u -m pytest tests/test_xgmi_gpu.py -x -v -k "collectives or dp_over or fsdp_over or fault" \
  --timeout 240 --timeout-method thread > gpurun_out/s3/pytest_xgmi.log 2>&1
rc=$?; echo "pytest xgmi rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/s3/pytest_xgmi.log | tail -20
[ $rc -ne 0 ] && { grep -E "Error|assert|Traceback" gpurun_out/s3/pytest_xgmi.log | head -20; exit $rc; }
timeout -k 10 600 python -u -m pytest tests/test_grad_scale_gpu.py -x -v -k "strategies" --timeout 240 \
  --timeout-method thread > gpurun_out/s3/pytest_scale.log 2>&1
rc=$?; echo "pytest grad-scale rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/s3/pytest_scale.log | tail -10
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/s3/pytest_scale.log | head -20; exit $rc; }
for cfg in "2 2" "2 4" "4 2"; do
  set -- $cfg
  timeout -k 10 180 python tools/stamp_xg_fsdp.py --ranks $1 --layers $2 > gpurun_out/s3/stamp_r$1_l$2.log 2>&1; rc=$?
  echo "== stamps ranks $1 layers $2 rc=$rc"; grep -v "amdgpu.ids\|socket.cpp\|Gloo" gpurun_out/s3/stamp_r$1_l$2.log | tail -8
  fatal $rc && exit $rc
done
export JDT_BACKEND=gloo
: > gpurun_out/s3/bench.jsonl
i=0
for rep in 1 2; do
  for cfg in "2|" "2|--strategy fsdp" "4|" "4|--strategy fsdp" "2|--num-layers 4" "2|--strategy fsdp --num-layers 4"; do
    n=${cfg%%|*}; a=${cfg#*|}; i=$((i+1))
    timeout -k 10 240 python bench.py --gpus $n --steps 200 --warmup 20 $a > gpurun_out/s3/b$i.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "N=$n '$a' rc=$rc"; grep -iE "error|timed" gpurun_out/s3/b$i.log | grep -v "^\[rank[1-9]" | tail -4; fatal $rc && exit $rc; continue; }
    echo "== rep $rep N=$n $a: $(grep '^{' gpurun_out/s3/b$i.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["details"]["collective_ms_p50"])')"
    grep '^{' gpurun_out/s3/b$i.log >> gpurun_out/s3/bench.jsonl
  done
done
unset JDT_BACKEND
bash tools/sessions/gpu_r4_hwq.sh
