#!/bin/bash
# Round 5 closing run 4 (final tree, after the md_bwd pin fix): the whole GPU suite and smoke(); every 1-GPU bench config; the driver
# form; headline phase stamps and rocprofv3 kernel stats; DP and FSDP at N = 2 / 4 / 8 ranks sharing
# the GPU (with their autotune tables); GPipe 2 / 4 stages; the entry scripts at 2 and 8 ranks
# with --check-replication.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5close4
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print(j["value"], j["ms_per_step"], c.get("step_launches", ""))'; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread \
  > gpurun_out/r5close4/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -3 gpurun_out/r5close4/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r5close4/pytest_gpu.log | head -20; fatal $rc && exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5close4/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/r5close4/smoke.log; exit 1; }
tail -1 gpurun_out/r5close4/smoke.log
: > gpurun_out/r5close4/all.jsonl
i=0
for a in "" "--optimizer sgd" "--num-layers 4" "--strategy fsdp" "--strategy fsdp --num-layers 4" \
         "--strategy pp --hidden-layers 8" "--strategy pp --model transformer" "--accum loop"; do
  i=$((i+1))
  timeout -k 10 180 python bench.py --steps 300 --warmup 30 $a > gpurun_out/r5close4/b$i.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "bench '$a' rc=$rc"; tail -5 gpurun_out/r5close4/b$i.log; fatal $rc && exit $rc; continue; }
  echo "== $a: $(js gpurun_out/r5close4/b$i.log)"
  grep '^{' gpurun_out/r5close4/b$i.log >> gpurun_out/r5close4/all.jsonl
done
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/r5close4/d$r.log 2>&1 || { tail -5 gpurun_out/r5close4/d$r.log; exit 1; }
  echo "== driver form $r: $(js gpurun_out/r5close4/d$r.log)"
done
timeout -k 10 120 python tools/stamp_pst.py --steps 200 --reps 3 > gpurun_out/r5close4/stamps.log 2>&1 || { echo stamps failed; tail -5 gpurun_out/r5close4/stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5close4/stamps.log | tail -12
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5close4/prof_h -o run -- \
  python3 bench.py --steps 400 --warmup 50 > gpurun_out/r5close4/prof_h.log 2>&1 || { tail -5 gpurun_out/r5close4/prof_h.log; exit 1; }
# N = 2 ranks sharing the GPU (gloo group; autotuned): the 2-layer and 4-layer DP / FSDP steps
for st in "" "--strategy fsdp" "--num-layers 4" "--strategy fsdp --num-layers 4"; do
  JDT_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 200 --warmup 20 $st > gpurun_out/r5close4/n2.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "N=2 '$st' rc=$rc"; tail -5 gpurun_out/r5close4/n2.log; exit $rc; }
  echo "== N=2 shared $st: $(js gpurun_out/r5close4/n2.log)"
  grep '^{' gpurun_out/r5close4/n2.log >> gpurun_out/r5close4/n2.jsonl
done
echo done
