#!/bin/bash
# Round 4 session 4: FSDP producer-staged collective (mlp2_bwd / md_bwd write the packed
# bucket; xg_fsdp_kernel skips phase 0): FSDP GPU tests at 2 / 8 ranks, stamps, N = 2 / 4
# A/B JDT_FSDP_STAGED=0/1 against DP; then the plain-torch hardware-queue reproducer LAST
# (GPU_MAX_HW_QUEUES=2, 4 graph branches: may crash, after which nothing else runs).
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s4
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -u -m pytest tests/test_xgmi_gpu.py -x -v -k "fsdp_over or collectives" \
  --timeout 240 --timeout-method thread > gpurun_out/s4/pytest_fsdp.log 2>&1
rc=$?; echo "pytest fsdp rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/s4/pytest_fsdp.log | tail -14
[ $rc -ne 0 ] && { grep -E "Error|assert|mismatch" gpurun_out/s4/pytest_fsdp.log | head -20; exit $rc; }
timeout -k 10 300 python -u -m pytest tests/test_rccl_capture_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/s4/pytest_rccl.log 2>&1 || { echo "rccl capture tests failed"; tail -20 gpurun_out/s4/pytest_rccl.log; exit 1; }
echo "rccl capture tests ok"
for cfg in "2 2" "2 4"; do
  set -- $cfg
  timeout -k 10 180 python tools/stamp_xg_fsdp.py --ranks $1 --layers $2 > gpurun_out/s4/stamp_r$1_l$2.log 2>&1; rc=$?
  echo "== stamps (staged) ranks $1 layers $2 rc=$rc"; grep -v "amdgpu.ids\|socket.cpp\|Gloo" gpurun_out/s4/stamp_r$1_l$2.log | tail -8
  fatal $rc && exit $rc
done
export JDT_BACKEND=gloo
: > gpurun_out/s4/bench.jsonl
i=0
for rep in 1 2; do
  for cfg in "2|1|--strategy fsdp" "2|0|--strategy fsdp" "2|1|" "4|1|--strategy fsdp" "4|0|--strategy fsdp" "4|1|" \
             "2|1|--strategy fsdp --num-layers 4" "2|0|--strategy fsdp --num-layers 4" "2|1|--num-layers 4"; do
    IFS='|' read n st a <<< "$cfg"; i=$((i+1))
    JDT_FSDP_STAGED=$st timeout -k 10 240 python bench.py --gpus $n --steps 200 --warmup 20 $a > gpurun_out/s4/b$i.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "N=$n staged=$st '$a' rc=$rc"; grep -iE "error|timed" gpurun_out/s4/b$i.log | grep -v "^\[rank[1-9]" | tail -4; fatal $rc && exit $rc; continue; }
    echo "== rep $rep N=$n staged=$st $a: $(grep '^{' gpurun_out/s4/b$i.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
    grep '^{' gpurun_out/s4/b$i.log >> gpurun_out/s4/bench.jsonl
  done
done
unset JDT_BACKEND
echo "== plain-torch reproducer, default hardware queues"
timeout -k 10 60 python tools/hwq_repro.py --streams 4 2>&1 | grep -v amdgpu.ids | tail -4
echo "== plain-torch reproducer, GPU_MAX_HW_QUEUES=2"
GPU_MAX_HW_QUEUES=2 timeout -k 10 60 python tools/hwq_repro.py --streams 4 > gpurun_out/s4/hwq_repro.log 2>&1; rc=$?
echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/s4/hwq_repro.log | head -14
