#!/bin/bash
# Round 4 session 5: full GPU suite + smoke on the round-4 tree, every 1-GPU bench config
# (regression check against round 3), driver form, headline phase stamps incl. the
# boundary between consecutive run-ahead launches.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s5
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/s5/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -3 gpurun_out/s5/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/s5/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s5/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/s5/smoke.log; exit 1; }
tail -1 gpurun_out/s5/smoke.log
: > gpurun_out/s5/all.jsonl
i=0
for a in "" "--optimizer sgd" "--num-layers 4" "--strategy fsdp" "--strategy fsdp --num-layers 4" \
         "--strategy pp --hidden-layers 8" "--strategy pp --model transformer" "--accum loop"; do
  i=$((i+1))
  timeout -k 10 180 python bench.py --steps 300 --warmup 30 $a > gpurun_out/s5/b$i.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "bench '$a' rc=$rc"; tail -5 gpurun_out/s5/b$i.log; fatal $rc && exit $rc; continue; }
  echo "== $a: $(grep '^{' gpurun_out/s5/b$i.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
  grep '^{' gpurun_out/s5/b$i.log >> gpurun_out/s5/all.jsonl
done
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/s5/default$r.log 2>&1 || { tail -5 gpurun_out/s5/default$r.log; exit 1; }
  echo "== driver form $r: $(grep '^{' gpurun_out/s5/default$r.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
done
timeout -k 10 120 python tools/stamp_mlp2.py > gpurun_out/s5/stamps.log 2>&1 || { echo stamps failed; tail -5 gpurun_out/s5/stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/s5/stamps.log | tail -45
echo done
