#!/bin/bash
# Round 4 session 19: the kernels without readfirstlane waterfall loops (md_bwd: wave index and
# step parity made scalar; the tile exchange: sys_rsrc_u) -- the deep / exchange / xGMI GPU tests,
# then the 1-GPU deep configs and the shared-GPU N = 2 one-launch steps (3 reps each).
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s19
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print(j["value"], j["ms_per_step"], c.get("step_launches", ""))'; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
  -k "deep or md_ or xgmi or tile_exchange or grad_scale or fused or stage or pipeline" > gpurun_out/s19/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/s19/pytest.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/s19/pytest.log | head -20; fatal $rc && exit $rc; exit 1; }
for r in 1 2 3; do
  for a in "--num-layers 4" "--strategy fsdp --num-layers 4" "--strategy pp --hidden-layers 8"; do
    timeout -k 10 120 python bench.py --steps 300 --warmup 30 $a > gpurun_out/s19/b.log 2>&1 || { echo "bench '$a' failed"; tail -5 gpurun_out/s19/b.log; exit 1; }
    echo "rep $r $a: $(js gpurun_out/s19/b.log)"
  done
  for a in "" "--strategy fsdp" "--num-layers 4"; do
    timeout -k 10 200 env JDT_BACKEND=gloo python bench.py --gpus 2 --steps 200 --warmup 20 $a > gpurun_out/s19/n.log 2>&1 || { echo "N=2 '$a' failed"; tail -5 gpurun_out/s19/n.log; exit 1; }
    echo "rep $r N=2 $a: $(js gpurun_out/s19/n.log)"
  done
  timeout -k 10 200 env JDT_BACKEND=gloo JDT_DP_DEEP_TX=1 python bench.py --gpus 2 --steps 200 --warmup 20 --num-layers 4 > gpurun_out/s19/n.log 2>&1 || { echo "N=2 deep tx failed"; tail -5 gpurun_out/s19/n.log; exit 1; }
  echo "rep $r N=2 --num-layers 4 JDT_DP_DEEP_TX=1: $(js gpurun_out/s19/n.log)"
done
echo done
