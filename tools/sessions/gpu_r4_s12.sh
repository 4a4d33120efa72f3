#!/bin/bash
# Round 4 session 12 (validation after the one-launch N > 1 work): the whole GPU suite,
# smoke(), every 1-GPU bench config, the driver form, and the DP headline at N = 2 / 4 / 8
# ranks sharing the GPU (2: one launch per step; 4 / 8: forward, backward, xGMI all-reduce).
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s12
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
  > gpurun_out/s12/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -3 gpurun_out/s12/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/s12/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s12/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/s12/smoke.log; exit 1; }
tail -1 gpurun_out/s12/smoke.log
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print(j["value"], j["ms_per_step"], c.get("step_launches", ""))'; }
: > gpurun_out/s12/all.jsonl
i=0
for a in "" "--optimizer sgd" "--num-layers 4" "--strategy fsdp" "--strategy fsdp --num-layers 4" \
         "--strategy pp --hidden-layers 8" "--strategy pp --model transformer" "--accum loop"; do
  i=$((i+1))
  timeout -k 10 180 python bench.py --steps 300 --warmup 30 $a > gpurun_out/s12/b$i.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "bench '$a' rc=$rc"; tail -5 gpurun_out/s12/b$i.log; fatal $rc && exit $rc; continue; }
  echo "== $a: $(js gpurun_out/s12/b$i.log)"
  grep '^{' gpurun_out/s12/b$i.log >> gpurun_out/s12/all.jsonl
done
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/s12/d$r.log 2>&1 || { tail -5 gpurun_out/s12/d$r.log; exit 1; }
  echo "== driver form $r: $(js gpurun_out/s12/d$r.log)"
done
for n in 2 4 8; do
  JDT_BACKEND=gloo timeout -k 10 300 python bench.py --gpus $n --steps 200 --warmup 20 > gpurun_out/s12/n$n.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "N=$n rc=$rc"; tail -5 gpurun_out/s12/n$n.log; fatal $rc && exit $rc; continue; }
  echo "== N=$n shared DP: $(js gpurun_out/s12/n$n.log)"
  grep '^{' gpurun_out/s12/n$n.log >> gpurun_out/s12/all.jsonl
done
echo done
