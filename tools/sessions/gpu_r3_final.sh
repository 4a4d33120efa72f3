#!/bin/bash
# Round-3 final: full GPU suite, every bench config on 1 GPU, the N = 2 / 4 shared-GPU
# rehearsals, and rocprofv3 kernel stats of the headline and transformer steps.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r3f
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r3f/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r3f/pytest_gpu.log
fatal $rc && exit $rc
: > gpurun_out/r3f/all.jsonl
i=0
for a in "" "--optimizer sgd" "--num-layers 4" "--num-layers 3" "--strategy fsdp" "--strategy fsdp --accum loop" \
         "--strategy pp --hidden-layers 8" "--strategy pp --model transformer" "--strategy pp --model transformer --microbatch-passes" \
         "--accum fused" "--accum loop" "--accum scan" "--strategy fsdp --num-layers 4"; do
  i=$((i+1))
  timeout -k 10 180 python bench.py --steps 300 --warmup 30 $a > gpurun_out/r3f/b$i.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "bench '$a' rc=$rc"; tail -5 gpurun_out/r3f/b$i.log; fatal $rc && exit $rc; continue; }
  echo "== $a: $(grep '^{' gpurun_out/r3f/b$i.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
  grep '^{' gpurun_out/r3f/b$i.log >> gpurun_out/r3f/all.jsonl
done
timeout -k 10 120 python bench.py > gpurun_out/r3f/default.log 2>&1 || { tail -5 gpurun_out/r3f/default.log; exit 1; }
echo "== default (driver form): $(grep '^{' gpurun_out/r3f/default.log)"
export JDT_BACKEND=gloo
for n in 2 4; do
  for a in "" "--strategy fsdp" "--strategy pp --hidden-layers 8" "--strategy pp --dp 2 --model transformer"; do
    [ "$a" = "--strategy pp --dp 2 --model transformer" ] && [ $n -ne 4 ] && continue
    i=$((i+1))
    timeout -k 10 240 python bench.py --gpus $n --steps 100 --warmup 10 $a > gpurun_out/r3f/b$i.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "N=$n '$a' rc=$rc"; tail -5 gpurun_out/r3f/b$i.log; fatal $rc && exit $rc; continue; }
    echo "== N=$n $a: $(grep '^{' gpurun_out/r3f/b$i.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); d=j["details"]; print(j["value"], j["ms_per_step"], d.get("comm"), d.get("step_launches"))')"
    grep '^{' gpurun_out/r3f/b$i.log >> gpurun_out/r3f/all.jsonl
  done
done
unset JDT_BACKEND
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3f/prof_head -o run -- \
  python3 bench.py --steps 300 --warmup 30 > gpurun_out/r3f/prof_head.log 2>&1 || exit 1
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3f/prof_lm -o run -- \
  python3 bench.py --strategy pp --model transformer --steps 100 --warmup 10 > gpurun_out/r3f/prof_lm.log 2>&1 || exit 1
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3f/prof_lmmb -o run -- \
  python3 bench.py --strategy pp --model transformer --microbatch-passes --steps 100 --warmup 10 > gpurun_out/r3f/prof_lmmb.log 2>&1 || exit 1
find gpurun_out/r3f -name "*kernel_stats.csv"
