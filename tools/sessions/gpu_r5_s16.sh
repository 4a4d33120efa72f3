#!/bin/bash
# Round 5 session 16: stage kernel + chip-wide AdamW launch
# one-launch-per-layer exchange (md_bwd FX): GPU tests + shared --gpus 2 bench with autotune.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s16
( while sleep 30; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 700 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_xgmi_gpu.py \
  tests/test_grad_scale_gpu.py -k "pipeline or stage_kernel" > gpurun_out/r5s16/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|Error|assert" gpurun_out/r5s16/pytest.log | head -40
fatal $rc && exit $rc
[ $rc -ne 0 ] && { grep -v amdgpu.ids gpurun_out/r5s16/pytest.log | tail -60; exit 1; }
export JDT_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 200 python tools/stamp_pp.py --gpus $n --microbatches 2 > gpurun_out/r5s16/stamp$n.log 2>&1; rc=$?
  grep -v -E "amdgpu.ids|Gloo|socket|connected peer" gpurun_out/r5s16/stamp$n.log | tail -14
  fatal $rc && exit $rc
done
for n in 2 4; do
  timeout -k 10 300 python bench.py --gpus $n --strategy pp --hidden-layers $n --steps 200 --warmup 20 > gpurun_out/r5s16/pp$n.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "pp$n rc=$rc"; grep -v amdgpu.ids gpurun_out/r5s16/pp$n.log | tail -15; fatal $rc && exit $rc; continue; }
  grep '^{' gpurun_out/r5s16/pp$n.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print("pp", c["parallelism"], j["value"], j["ms_per_step"], c.get("num_microbatches"), c.get("step_launches",""), json.dumps(j["details"].get("autotune"))[:800])'
done
