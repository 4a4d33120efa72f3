#!/bin/bash
# Round 5 session 2: the whole GPU suite (autotune validation / fallback rehearsals, the
# input-width-1024 fused engine at N = 1 and 2 shared ranks, no 8-rank skip), smoke() with
# its numeric check, the driver-form headline, BASELINE config #3's layout at 8 shared
# ranks three times, and the 4-layer DP / FSDP at 2 shared ranks with their autotune tables.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s2
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rs --durations=15 --timeout 300 --timeout-method thread \
  > gpurun_out/r5s2/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; grep -E "passed|failed|SKIP|FAILED|Error" gpurun_out/r5s2/pytest_gpu.log | tail -30
fatal $rc && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5s2/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/r5s2/smoke.log; exit 1; }
tail -1 gpurun_out/r5s2/smoke.log
for r in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/r5s2/d$r.log 2>&1 || { tail -5 gpurun_out/r5s2/d$r.log; exit 1; }
  grep '^{' gpurun_out/r5s2/d$r.log | cut -c1-300
done
export JDT_BACKEND=gloo
for st in dp fsdp; do
  timeout -k 10 300 python bench.py --gpus 2 --steps 200 --warmup 20 --strategy $st --num-layers 4 > gpurun_out/r5s2/n2l4_$st.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { tail -20 gpurun_out/r5s2/n2l4_$st.log; fatal $rc && exit $rc; continue; }
  grep '^{' gpurun_out/r5s2/n2l4_$st.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["config"]["parallelism"], j["value"], j["config"].get("step_launches"), json.dumps(j["details"]["autotune"])[:600])'
done
for r in 1 2 3; do
  timeout -k 10 400 python bench.py --gpus 8 --strategy fsdp --num-layers 4 --steps 100 --warmup 10 > gpurun_out/r5s2/f8l4_$r.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "fsdp8 4-layer run $r rc=$rc"; tail -20 gpurun_out/r5s2/f8l4_$r.log; fatal $rc && exit $rc; continue; }
  grep '^{' gpurun_out/r5s2/f8l4_$r.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print("fsdp8 4-layer run", j["value"], j["ms_per_step"])'
done
