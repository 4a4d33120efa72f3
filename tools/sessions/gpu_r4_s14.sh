#!/bin/bash
# Round 4 session 14: the one-launch N > 1 FSDP step (partials to their rows' owners, sharded
# AdamW in the kernel, updated values handed back): the FSDP / DP xGMI tests and the
# grad-scale probes, then shared-GPU FSDP2 A/B (JDT_FSDP_AHEAD 1 / 0) next to DP2.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s14
timeout -k 10 700 python -u -m pytest tests/test_xgmi_gpu.py tests/test_grad_scale_gpu.py -m gpu -v --timeout 240 \
  --timeout-method thread -k "fsdp" > gpurun_out/s14/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|SKIPPED" gpurun_out/s14/pytest.log | tail -30
[ $rc -ne 0 ] && { grep -E "Error|assert|timed out|error word" gpurun_out/s14/pytest.log | head -30; exit $rc; }
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print(j["value"], j["ms_per_step"], c.get("step_launches", ""))'; }
run() {
  timeout -k 10 200 env $2 python bench.py $3 > gpurun_out/s14/b.log 2>&1 || { echo "bench $1 failed"; tail -8 gpurun_out/s14/b.log; exit 1; }
  echo "$1: $(js gpurun_out/s14/b.log)"
}
for r in 1 2 3; do
  run "rep $r N=2 FSDP one-launch" "JDT_BACKEND=gloo JDT_FSDP_AHEAD=1" "--gpus 2 --strategy fsdp --steps 200 --warmup 20"
  run "rep $r N=2 FSDP three-launch" "JDT_BACKEND=gloo JDT_FSDP_AHEAD=0" "--gpus 2 --strategy fsdp --steps 200 --warmup 20"
  run "rep $r N=2 DP one-launch" "JDT_BACKEND=gloo" "--gpus 2 --steps 200 --warmup 20"
done
timeout -k 10 300 python param_sharding.py --gpus 2 --check-replication > gpurun_out/s14/e.log 2>&1 || { tail -8 gpurun_out/s14/e.log; exit 1; }
echo "param_sharding.py --gpus 2 --check-replication:"; grep -iE "replicat|loss|accuracy" gpurun_out/s14/e.log | tail -3
echo done
