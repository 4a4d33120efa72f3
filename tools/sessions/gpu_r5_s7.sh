#!/bin/bash
# Round 5 session 7: GPipe stage kernel with dZ hops (predecessor forms dH from the
# successor's weight image): pipeline GPU tests, sub-tick stamps, GPipe bench.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s7
( while sleep 30; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_xgmi_gpu.py \
  -k "pipeline" > gpurun_out/r5s7/pytest_pp.log 2>&1
rc=$?; echo "pytest pp rc=$rc"; grep -E "PASSED|FAILED|Error|assert" gpurun_out/r5s7/pytest_pp.log | head -30
fatal $rc && exit $rc
[ $rc -ne 0 ] && { grep -v amdgpu.ids gpurun_out/r5s7/pytest_pp.log | tail -60; exit 1; }
export JDT_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 200 python tools/stamp_pp.py --gpus $n --microbatches 4 > gpurun_out/r5s7/stamp$n.log 2>&1; rc=$?
  grep -v -E "amdgpu.ids|Gloo|socket|connected peer" gpurun_out/r5s7/stamp$n.log | tail -14
  fatal $rc && exit $rc
done
for n in 2 4; do
  timeout -k 10 300 python bench.py --gpus $n --strategy pp --hidden-layers $n --steps 200 --warmup 20 > gpurun_out/r5s7/pp$n.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "pp$n rc=$rc"; grep -v amdgpu.ids gpurun_out/r5s7/pp$n.log | tail -15; fatal $rc && exit $rc; continue; }
  grep '^{' gpurun_out/r5s7/pp$n.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print("pp", c["parallelism"], j["value"], j["ms_per_step"], c.get("num_microbatches"), c.get("step_launches",""), json.dumps(j["details"].get("autotune"))[:1500])'
done
