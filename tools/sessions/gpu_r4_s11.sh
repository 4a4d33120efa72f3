#!/bin/bash
# Round 4 session 11: the deep engine's N > 1 step with every hidden layer's backward
# exchanging its gradient tiles in-kernel (layer 0 running ahead): DP at ws = 2 (2- and
# 4-layer, one-launch and three-launch) equal to one device, the exchange self-test; then
# shared-GPU A/B at N = 2 (4-layer and 2-layer, JDT_DP_AHEAD 1 / 0) and the 1-GPU 4-layer.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s11
timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py tests/test_grad_scale_gpu.py -m gpu -v -s --timeout 240 \
  --timeout-method thread -k "dp_over_xgmi or dp_adam or dp4_adam or dp_sgd" > gpurun_out/s11/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|\[dp ws" gpurun_out/s11/pytest.log | tail -30
[ $rc -ne 0 ] && { grep -E "Error|assert|timed out|error word" gpurun_out/s11/pytest.log | head -30; exit $rc; }
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print(j["value"], j["ms_per_step"], c.get("step_launches"))'; }
run() {
  timeout -k 10 200 env $2 python bench.py $3 > gpurun_out/s11/b.log 2>&1 || { echo "bench $1 failed"; tail -8 gpurun_out/s11/b.log; exit 1; }
  echo "$1: $(js gpurun_out/s11/b.log)"
}
for r in 1 2; do
  run "rep $r N=2 4-layer DP exchange" "JDT_BACKEND=gloo JDT_DP_AHEAD=1" "--gpus 2 --num-layers 4 --steps 200 --warmup 20"
  run "rep $r N=2 4-layer DP three-launch-style" "JDT_BACKEND=gloo JDT_DP_AHEAD=0" "--gpus 2 --num-layers 4 --steps 200 --warmup 20"
  run "rep $r N=2 2-layer DP one-launch" "JDT_BACKEND=gloo" "--gpus 2 --steps 200 --warmup 20"
  run "rep $r N=1 4-layer" "" "--num-layers 4 --steps 300 --warmup 30"
done
echo done
