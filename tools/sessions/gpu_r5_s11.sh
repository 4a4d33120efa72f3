#!/bin/bash
# Round 5 session 11: benches on the shared GPU (gloo bootstrap): GPipe 2 / 4 stages with
# the 8-wave stage kernel; 4-layer FSDP and DP at --gpus 2 with their autotune tables.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 JDT_BACKEND=gloo && mkdir -p gpurun_out/r5s11
( while sleep 30; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
show() { grep '^{' "$1" | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print(c["parallelism"], c.get("model",""), j["value"], j["ms_per_step"], c.get("num_microbatches",""), c.get("step_launches",""), json.dumps(j["details"].get("autotune"))[:1200])'; }
for n in 2 4; do
  timeout -k 10 300 python bench.py --gpus $n --strategy pp --hidden-layers $n --steps 200 --warmup 20 > gpurun_out/r5s11/pp$n.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "pp$n rc=$rc"; grep -v amdgpu.ids gpurun_out/r5s11/pp$n.log | tail -15; fatal $rc && exit $rc; continue; }
  show gpurun_out/r5s11/pp$n.log
done
for s in fsdp dp; do
  timeout -k 10 300 python bench.py --gpus 2 --strategy $s --num-layers 4 --steps 300 --warmup 20 > gpurun_out/r5s11/${s}4.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "${s}4 rc=$rc"; grep -v amdgpu.ids gpurun_out/r5s11/${s}4.log | tail -15; fatal $rc && exit $rc; continue; }
  show gpurun_out/r5s11/${s}4.log
done
