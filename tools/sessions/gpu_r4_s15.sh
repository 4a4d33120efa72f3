#!/bin/bash
# Round 4 session 15: validation after the one-launch FSDP step -- the whole GPU suite, smoke(),
# the headline (300 steps, 3 reps), shared-GPU FSDP2 / DP2 one launch, and param_sharding.py at
# 2 ranks (FSDP one launch) with --check-replication.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s15
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print(j["value"], j["ms_per_step"], c.get("step_launches", ""))'; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
  > gpurun_out/s15/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -3 gpurun_out/s15/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/s15/pytest_gpu.log | head -20; fatal $rc && exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s15/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/s15/smoke.log; exit 1; }
tail -1 gpurun_out/s15/smoke.log
for r in 1 2 3; do
  timeout -k 10 180 python bench.py --steps 300 --warmup 30 > gpurun_out/s15/h$r.log 2>&1 || { tail -5 gpurun_out/s15/h$r.log; exit 1; }
  echo "== headline $r: $(js gpurun_out/s15/h$r.log)"
done
export JDT_BACKEND=gloo
for a in "--strategy fsdp" ""; do
  timeout -k 10 300 python bench.py --gpus 2 --steps 200 --warmup 20 $a > gpurun_out/s15/n2.log 2>&1 || { tail -5 gpurun_out/s15/n2.log; exit 1; }
  echo "== N=2 $a: $(js gpurun_out/s15/n2.log)"
done
timeout -k 10 300 python param_sharding.py --gpus 2 --check-replication > gpurun_out/s15/e.log 2>&1 || { tail -8 gpurun_out/s15/e.log; exit 1; }
echo "== param_sharding.py --gpus 2 --check-replication:"; grep -iE "replicat|loss|accuracy|one.launch" gpurun_out/s15/e.log | tail -4
echo done
