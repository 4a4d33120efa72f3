#!/bin/bash
# Round 5 session 20: after the stage-body refactor (inlined device function, carved LDS):
# the pipeline / stage-kernel / chain GPU tests and the PP2 / PP4 benches.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s20
( while sleep 30; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 700 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_xgmi_gpu.py tests/test_grad_scale_gpu.py \
  tests/test_pp_chain_gpu.py -k "pipeline or stage_kernel or chain" > gpurun_out/r5s20/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/r5s20/pytest.log | tail -8
fatal $rc && exit $rc
export JDT_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 300 python bench.py --gpus $n --strategy pp --hidden-layers $n --steps 200 --warmup 20 > gpurun_out/r5s20/pp$n.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "pp$n rc=$rc"; tail -15 gpurun_out/r5s20/pp$n.log; fatal $rc && exit $rc; continue; }
  grep '^{' gpurun_out/r5s20/pp$n.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print("pp", c["parallelism"], j["value"], j["ms_per_step"], c.get("num_microbatches"), c.get("step_launches",""))'
done
