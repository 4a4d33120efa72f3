#!/bin/bash
# Round 4 session 9: the one-launch N > 1 DP step (run-ahead backward with the in-kernel
# per-tile gradient exchange, comm/tile_exchange.py): correctness at ws = 2 (shared GPU;
# 2 x 224 workgroups fit), the three-launch fallback at ws = 2 / 8, grad-scale probes;
# then shared-GPU DP2 A/B (JDT_DP_AHEAD 1 / 0) and the 1-GPU headline after the phase-3
# restructure.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s9
timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py tests/test_grad_scale_gpu.py -m gpu -x -v --timeout 240 \
  --timeout-method thread -k "dp_over_xgmi or collectives or dp" > gpurun_out/s9/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/s9/pytest.log | tail -30
[ $rc -ne 0 ] && { grep -E "Error|assert|timed out|error word" gpurun_out/s9/pytest.log | head -30; exit $rc; }
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print(j["value"], j["ms_per_step"], c.get("step_launches"))'; }
run() {
  timeout -k 10 200 env $2 python bench.py $3 > gpurun_out/s9/b.log 2>&1 || { echo "bench $1 failed"; tail -8 gpurun_out/s9/b.log; exit 1; }
  echo "$1: $(js gpurun_out/s9/b.log)"
}
for r in 1 2 3; do
  run "rep $r N=2 DP one-launch" "JDT_BACKEND=gloo JDT_DP_AHEAD=1" "--gpus 2 --steps 200 --warmup 20"
  run "rep $r N=2 DP three-launch" "JDT_BACKEND=gloo JDT_DP_AHEAD=0" "--gpus 2 --steps 200 --warmup 20"
  run "rep $r N=1 headline" "" "--steps 300 --warmup 30"
done
run "N=2 DP one-launch driver form" "JDT_BACKEND=gloo" "--gpus 2 --steps 20 --warmup 5"
echo done
