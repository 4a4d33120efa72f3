#!/bin/bash
# Round 5 session 1: the whole GPU suite on a fresh box with skip reasons and the slowest
# tests (incl. the autotune validation / fallback rehearsals), the driver-form headline
# bench, and the 2-rank shared-GPU DP / FSDP benches with their autotune tables.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rs --durations=30 --timeout 240 --timeout-method thread \
  > gpurun_out/r5s1/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; grep -E "passed|failed|SKIP|FAILED" gpurun_out/r5s1/pytest_gpu.log | tail -30
case $rc in 124|134|137|139) exit $rc;; esac
for r in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/r5s1/d$r.log 2>&1 || { tail -5 gpurun_out/r5s1/d$r.log; exit 1; }
  grep '^{' gpurun_out/r5s1/d$r.log | cut -c1-400
done
export JDT_BACKEND=gloo
for st in dp fsdp; do
  timeout -k 10 300 python bench.py --gpus 2 --steps 200 --warmup 20 --strategy $st > gpurun_out/r5s1/n2_$st.log 2>&1 || { tail -20 gpurun_out/r5s1/n2_$st.log; exit 1; }
  grep '^{' gpurun_out/r5s1/n2_$st.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["config"].get("step_launches"), json.dumps(j["details"]["autotune"]))'
done
