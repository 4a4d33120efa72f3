#!/bin/bash
# Round-3 closing run: full GPU suite + smoke, every bench config on 1 GPU (incl. the stream
# schedules), driver form, N = 2 / 4 shared-GPU rehearsals (incl. DP2 x one-stage LM on streams),
# entry scripts, rocprofv3 stats of the headline and the LM default step.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/f2
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/f2/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/f2/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/f2/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/f2/smoke.log; exit 1; }
tail -1 gpurun_out/f2/smoke.log
: > gpurun_out/f2/all.jsonl
i=0
for a in "" "--optimizer sgd" "--num-layers 4" "--num-layers 3" "--strategy fsdp" "--strategy fsdp --accum loop" \
         "--strategy pp --hidden-layers 8" "--strategy pp --model transformer" "--accum fused" "--accum loop" \
         "--accum loop --num-layers 4" "--accum scan" "--strategy fsdp --num-layers 4"; do
  i=$((i+1))
  timeout -k 10 180 python bench.py --steps 300 --warmup 30 $a > gpurun_out/f2/b$i.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "bench '$a' rc=$rc"; tail -5 gpurun_out/f2/b$i.log; fatal $rc && exit $rc; continue; }
  echo "== $a: $(grep '^{' gpurun_out/f2/b$i.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
  grep '^{' gpurun_out/f2/b$i.log >> gpurun_out/f2/all.jsonl
done
JDT_MB_STREAMS=1 timeout -k 10 180 python bench.py --steps 300 --warmup 30 --strategy pp --model transformer > gpurun_out/f2/lm1.log 2>&1 || exit 1
echo "== LM JDT_MB_STREAMS=1 (layer-major): $(grep '^{' gpurun_out/f2/lm1.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["config"]["single_stage_mode"])')"
grep '^{' gpurun_out/f2/lm1.log >> gpurun_out/f2/all.jsonl
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/f2/default.log 2>&1 || { tail -5 gpurun_out/f2/default.log; exit 1; }
echo "== driver form: $(grep '^{' gpurun_out/f2/default.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
export JDT_BACKEND=gloo
for cfg in "2|" "4|" "2|--strategy fsdp" "4|--strategy pp --hidden-layers 8" "2|--strategy pp --dp 2 --model transformer" "4|--strategy pp --dp 2 --model transformer"; do
  n=${cfg%%|*}; a=${cfg#*|}
  i=$((i+1))
  timeout -k 10 240 python bench.py --gpus $n --steps 100 --warmup 10 $a > gpurun_out/f2/b$i.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "N=$n '$a' rc=$rc"; tail -5 gpurun_out/f2/b$i.log; fatal $rc && exit $rc; continue; }
  echo "== N=$n $a: $(grep '^{' gpurun_out/f2/b$i.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["config"].get("single_stage_mode"))')"
  grep '^{' gpurun_out/f2/b$i.log >> gpurun_out/f2/all.jsonl
done
unset JDT_BACKEND
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f2/prof_head -o run -- \
  python3 bench.py --steps 300 --warmup 30 > gpurun_out/f2/prof_head.log 2>&1 || exit 1
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f2/prof_loop4 -o run -- \
  python3 bench.py --accum loop --num-layers 4 --steps 100 --warmup 10 > gpurun_out/f2/prof_loop4.log 2>&1 || exit 1
echo done
