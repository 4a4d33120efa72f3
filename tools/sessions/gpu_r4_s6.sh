#!/bin/bash
# Round 4 session 6: write-through (sc1) stores of the AdamW state in the run-ahead
# mlp2_bwd (JDT_MLP2_WT: 1 = p/m/v + W1^T, 3 = + Z1 partials and G1) and in md_bwd
# (JDT_MD_WT=1), so the kernel boundary has fewer dirty L2 lines to write back.
# Correctness with them on, then alternating A/B (300 steps), then headline stamps.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s6
JDT_MLP2_WT=3 JDT_MD_WT=1 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_grad_scale_gpu.py \
  -m gpu -x -q --timeout 120 --timeout-method thread -k "ahead or deep or mlp2 or fused or scale" \
  > gpurun_out/s6/pytest_wt.log 2>&1
rc=$?; echo "pytest (wt on) rc=$rc"; tail -3 gpurun_out/s6/pytest_wt.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/s6/pytest_wt.log | head -20; exit $rc; }
run() {  # label, env, args
  timeout -k 10 120 env $2 python bench.py --steps 300 --warmup 30 $3 > gpurun_out/s6/b.log 2>&1 || { echo "bench $1 failed"; tail -5 gpurun_out/s6/b.log; exit 1; }
  echo "$1: $(grep '^{' gpurun_out/s6/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
}
for r in 1 2 3; do
  run "rep $r headline wt=0" "JDT_MLP2_WT=0" ""
  run "rep $r headline wt=1" "JDT_MLP2_WT=1" ""
  run "rep $r headline wt=3" "JDT_MLP2_WT=3" ""
  run "rep $r 4-layer md_wt=0" "JDT_MD_WT=0" "--num-layers 4"
  run "rep $r 4-layer md_wt=1" "JDT_MD_WT=1" "--num-layers 4"
done
for r in 1 2; do
  run "rep $r pp8 md_wt=0" "JDT_MD_WT=0" "--strategy pp --hidden-layers 8"
  run "rep $r pp8 md_wt=1" "JDT_MD_WT=1" "--strategy pp --hidden-layers 8"
done
# per-part data-axis sync overlapping the W pass (pipeline._overlapped_sync): tests, then
# DP2 x PP2 LM (4 ranks sharing the GPU) A/B
timeout -k 10 400 python -u -m pytest tests/test_xgmi_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "collectives or transformer_hybrid" > gpurun_out/s6/pytest_xg.log 2>&1
rc=$?; echo "pytest xgmi (overlap sync) rc=$rc"; tail -3 gpurun_out/s6/pytest_xg.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/s6/pytest_xg.log | head -20; exit $rc; }
for r in 1 2; do
  for ov in 1 0; do
    JDT_BACKEND=gloo JDT_PP_OVERLAP_SYNC=$ov timeout -k 10 200 python bench.py --gpus 4 --strategy pp --dp 2 --model transformer \
      --steps 60 --warmup 10 > gpurun_out/s6/lm$ov.log 2>&1 || { echo "lm bench ov=$ov failed"; tail -5 gpurun_out/s6/lm$ov.log; exit 1; }
    echo "rep $r DP2xPP2 LM overlap_sync=$ov: $(grep '^{' gpurun_out/s6/lm$ov.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
  done
done
for wt in 0 3; do
  JDT_MLP2_WT=$wt timeout -k 10 120 python tools/stamp_mlp2.py > gpurun_out/s6/stamps_wt$wt.log 2>&1 || { echo stamps failed; tail -5 gpurun_out/s6/stamps_wt$wt.log; exit 1; }
  echo "--- stamps wt=$wt"; grep -E "run-ahead|span|column barrier|Z1 partial|dW1" gpurun_out/s6/stamps_wt$wt.log | tail -8
done
echo done
