#!/bin/bash
# Round 4 session 22: the FSDP one-launch partial stores through uniform per-owner resources
# (no waterfall loop left in any kernel): FSDP / exchange GPU tests, then shared-GPU FSDP2 (3 reps).
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s22
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print(j["value"], j["ms_per_step"], c.get("step_launches", ""))'; }
timeout -k 10 700 python -u -m pytest tests/test_xgmi_gpu.py tests/test_grad_scale_gpu.py tests/test_bench_fallback_gpu.py -m gpu -q \
  --timeout 300 --timeout-method thread -k "fsdp or tile_exchange" > gpurun_out/s22/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/s22/pytest.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/s22/pytest.log | head -20; fatal $rc && exit $rc; exit 1; }
for r in 1 2 3; do
  timeout -k 10 200 env JDT_BACKEND=gloo python bench.py --gpus 2 --steps 200 --warmup 20 --strategy fsdp > gpurun_out/s22/n.log 2>&1 || { echo "N=2 fsdp failed"; tail -5 gpurun_out/s22/n.log; exit 1; }
  echo "rep $r N=2 fsdp: $(js gpurun_out/s22/n.log)"
done
timeout -k 10 300 env JDT_BACKEND=gloo python param_sharding.py --gpus 2 --check-replication > gpurun_out/s22/e.log 2>&1 || { tail -8 gpurun_out/s22/e.log; exit 1; }
grep -iE "replicat|loss|accuracy" gpurun_out/s22/e.log | tail -3
echo done
