#!/bin/bash
# Round 5 session 19: the one-GPU chain (every MLP layer a stage of one launch): its GPU
# tests, then the one-GPU GPipe benches (8 and 4 hidden layers) with and without it.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s19
( while sleep 30; do echo "[hb] $(date +%T)"; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_pp_chain_gpu.py \
  > gpurun_out/r5s19/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|Error|assert" gpurun_out/r5s19/pytest.log | head -20
fatal $rc && exit $rc
[ $rc -ne 0 ] && { grep -v amdgpu.ids gpurun_out/r5s19/pytest.log | tail -50; exit 1; }
for L in 8 4; do for k in 1 0; do for n in 4 2; do
  JDT_PP_KERNEL=$k timeout -k 10 200 python bench.py --strategy pp --hidden-layers $L --microbatches $n --steps 300 --warmup 30 \
    > gpurun_out/r5s19/pp1_L${L}_k${k}_n$n.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "L$L k$k n$n rc=$rc"; tail -8 gpurun_out/r5s19/pp1_L${L}_k${k}_n$n.log; fatal $rc && exit $rc; continue; }
  grep '^{' gpurun_out/r5s19/pp1_L${L}_k${k}_n$n.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print("L'$L' kernel='$k' n='$n'", j["value"], j["ms_per_step"], c.get("step_launches",""))'
done; done; done
