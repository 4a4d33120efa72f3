#!/bin/bash
# Round 4 closing run 2 (after the one-launch FSDP step, the bench fallback and the waterfall-free kernels): the whole GPU suite and smoke(); every 1-GPU bench config; the driver
# form; headline phase stamps (incl. the boundary between run-ahead launches) and rocprofv3
# kernel stats; the DP headline at N = 2 / 4 / 8 ranks sharing the GPU; the entry scripts at
# 2 ranks (DP: one launch per step) and at 8 ranks, each with --check-replication.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/close2
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print(j["value"], j["ms_per_step"], c.get("step_launches", ""))'; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
  > gpurun_out/close2/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -3 gpurun_out/close2/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/close2/pytest_gpu.log | head -20; fatal $rc && exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/close2/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/close2/smoke.log; exit 1; }
tail -1 gpurun_out/close2/smoke.log
: > gpurun_out/close2/all.jsonl
i=0
for a in "" "--optimizer sgd" "--num-layers 4" "--strategy fsdp" "--strategy fsdp --num-layers 4" \
         "--strategy pp --hidden-layers 8" "--strategy pp --model transformer" "--accum loop"; do
  i=$((i+1))
  timeout -k 10 180 python bench.py --steps 300 --warmup 30 $a > gpurun_out/close2/b$i.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "bench '$a' rc=$rc"; tail -5 gpurun_out/close2/b$i.log; fatal $rc && exit $rc; continue; }
  echo "== $a: $(js gpurun_out/close2/b$i.log)"
  grep '^{' gpurun_out/close2/b$i.log >> gpurun_out/close2/all.jsonl
done
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/close2/d$r.log 2>&1 || { tail -5 gpurun_out/close2/d$r.log; exit 1; }
  echo "== driver form $r: $(js gpurun_out/close2/d$r.log)"
done
timeout -k 10 120 python tools/stamp_mlp2.py > gpurun_out/close2/stamps.log 2>&1 || { echo stamps failed; tail -5 gpurun_out/close2/stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/close2/stamps.log | tail -12
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/close2/prof_h -o run -- \
  python3 bench.py --steps 400 --warmup 50 > gpurun_out/close2/prof_h.log 2>&1 || { tail -5 gpurun_out/close2/prof_h.log; exit 1; }
export JDT_BACKEND=gloo
for n in 2 4 8; do for st in "" "--strategy fsdp"; do
  timeout -k 10 300 python bench.py --gpus $n --steps 200 --warmup 20 $st > gpurun_out/close2/n$n.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "N=$n rc=$rc"; tail -5 gpurun_out/close2/n$n.log; fatal $rc && exit $rc; continue; }
  echo "== N=$n shared $st: $(js gpurun_out/close2/n$n.log)"
  grep '^{' gpurun_out/close2/n$n.log >> gpurun_out/close2/all.jsonl
done; done
for s in "data_paral.py --gpus 2" "param_sharding.py --gpus 2" "data_paral.py --gpus 8 --num-layers 4" "param_sharding.py --gpus 8 --num-layers 4" \
         "pipeline_parallel.py --gpus 8" "pipeline_parallel.py --gpus 8 --dp 2 --model transformer"; do
  i=$((i+1))
  timeout -k 10 300 python $s --check-replication > gpurun_out/close2/e$i.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "entry '$s' rc=$rc"; tail -8 gpurun_out/close2/e$i.log; fatal $rc && exit $rc; continue; }
  echo "== entry $s --check-replication:"; grep -iE "replicat|loss|accuracy" gpurun_out/close2/e$i.log | tail -3
done
echo done
