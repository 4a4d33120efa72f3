#!/bin/bash
# Round 5 session 12: the autotune with the candidate env in force through its validation
# steps (the fix): the bench fallback / corruption tests, then 2-layer and 4-layer DP / FSDP
# at --gpus 2 on the shared GPU with their autotune tables (validation errors between forms).
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s12
( while sleep 30; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bench_fallback_gpu.py \
  > gpurun_out/r5s12/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|Error|assert" gpurun_out/r5s12/pytest.log | head -20
fatal $rc && exit $rc
[ $rc -ne 0 ] && { grep -v amdgpu.ids gpurun_out/r5s12/pytest.log | tail -60; exit 1; }
export JDT_BACKEND=gloo
show() { grep '^{' "$1" | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print(c["parallelism"], c.get("model","")[:30], j["value"], j["ms_per_step"], c.get("step_launches",""), json.dumps(j["details"].get("autotune"))[:1500])'; }
for L in 2 4; do for s in dp fsdp; do
  timeout -k 10 300 python bench.py --gpus 2 --strategy $s --num-layers $L --steps 300 --warmup 20 > gpurun_out/r5s12/${s}$L.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "${s}$L rc=$rc"; grep -v amdgpu.ids gpurun_out/r5s12/${s}$L.log | tail -15; fatal $rc && exit $rc; continue; }
  show gpurun_out/r5s12/${s}$L.log
done; done
