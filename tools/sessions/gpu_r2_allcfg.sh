#!/bin/bash
# Round-2 table: every bench config on 1 GPU (300 steps), then the N = 2 / 4 paths with
# ranks sharing the one GPU (built-in launcher, gloo bootstrap, xGMI kernels between processes)
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/all
: > gpurun_out/all/r2_all.jsonl
i=0
for a in "" "--optimizer sgd" "--num-layers 4" "--num-layers 3" "--strategy fsdp" "--strategy fsdp --num-layers 4" \
         "--strategy pp --hidden-layers 8" "--strategy pp --model transformer" "--strategy pp --model transformer --merge-microbatches" \
         "--accum fused" "--accum loop" "--accum scan"; do
  i=$((i+1))
  timeout -k 10 180 python bench.py --steps 300 --warmup 30 $a > gpurun_out/all/b$i.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "bench '$a' rc=$rc"; tail -5 gpurun_out/all/b$i.log; exit $rc; }
  echo "== $a: $(grep '^{' gpurun_out/all/b$i.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
  grep '^{' gpurun_out/all/b$i.log >> gpurun_out/all/r2_all.jsonl
done
export JDT_BACKEND=gloo
for n in 2 4; do
  for a in "" "--strategy fsdp" "--strategy pp --hidden-layers 8" "--strategy pp --dp 2 --model transformer"; do
    [ "$a" = "--strategy pp --dp 2 --model transformer" ] && [ $n -ne 4 ] && continue
    i=$((i+1))
    timeout -k 10 240 python bench.py --gpus $n --steps 100 --warmup 10 $a > gpurun_out/all/b$i.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "N=$n '$a' rc=$rc"; tail -5 gpurun_out/all/b$i.log; exit $rc; }
    echo "== N=$n $a: $(grep '^{' gpurun_out/all/b$i.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["details"].get("comm"), j["details"].get("xgmi_selftest"))')"
    grep '^{' gpurun_out/all/b$i.log >> gpurun_out/all/r2_all.jsonl
  done
done
