#!/bin/bash
# Round 5 session 3: BASELINE config #3's layout (--gpus 8 --strategy fsdp --num-layers 4)
# three times on the shared GPU with the xGMI grids capped for 8 sharing ranks; then the
# 8-rank DP / GPipe-8 / DP2 x PP4 LM benches with their autotune tables.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 JDT_BACKEND=gloo && mkdir -p gpurun_out/r5s3
( while sleep 30; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
summ() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print(c["parallelism"], j["value"], j["ms_per_step"], c.get("num_microbatches"), c.get("step_launches",""), json.dumps(j["details"].get("autotune"))[:900])'; }
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 8 --strategy fsdp --num-layers 4 --steps 100 --warmup 10 > gpurun_out/r5s3/f8l4_$r.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "fsdp8 4-layer run $r rc=$rc"; grep -v amdgpu.ids gpurun_out/r5s3/f8l4_$r.log | tail -15; fatal $rc && exit $rc; continue; }
  echo "== fsdp8 4-layer run $r: $(summ gpurun_out/r5s3/f8l4_$r.log)"
done
for a in "" "--num-layers 4" "--strategy pp --hidden-layers 8" "--strategy pp --model transformer --dp 2"; do
  timeout -k 10 400 python bench.py --gpus 8 --steps 100 --warmup 10 $a > gpurun_out/r5s3/b8.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "8 ranks '$a' rc=$rc"; grep -v amdgpu.ids gpurun_out/r5s3/b8.log | tail -15; fatal $rc && exit $rc; continue; }
  echo "== 8 ranks $a: $(summ gpurun_out/r5s3/b8.log)"
  grep '^{' gpurun_out/r5s3/b8.log >> gpurun_out/r5s3/all.jsonl
done
