#!/bin/bash
# Round 4 session 7: (a) the overlapped per-GEMM data-axis sync of multi-stage pipelines and
# the xGMI kernels' write-through AdamW stores (JDT_XG_WT=1) under the xGMI GPU tests;
# (b) shared-GPU A/B: DP2 / DP4 / FSDP2 with JDT_XG_WT 0/1, DP2 x PP2 LM with
# JDT_PP_OVERLAP_SYNC 0/1; (c) 1-GPU headline and 4-layer with the new write-through defaults.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s7
JDT_XG_WT=1 timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/s7/pytest_xg.log 2>&1
rc=$?; echo "pytest test_xgmi_gpu (JDT_XG_WT=1) rc=$rc"; tail -3 gpurun_out/s7/pytest_xg.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/s7/pytest_xg.log | head -20; exit $rc; }
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])'; }
run() {  # label, env, args
  timeout -k 10 200 env $2 python bench.py $3 > gpurun_out/s7/b.log 2>&1 || { echo "bench $1 failed"; tail -5 gpurun_out/s7/b.log; exit 1; }
  echo "$1: $(js gpurun_out/s7/b.log)"
}
for r in 1 2; do
  for wt in 0 1; do
    run "rep $r N=2 DP xg_wt=$wt" "JDT_BACKEND=gloo JDT_XG_WT=$wt" "--gpus 2 --steps 200 --warmup 20"
    run "rep $r N=2 FSDP xg_wt=$wt" "JDT_BACKEND=gloo JDT_XG_WT=$wt" "--gpus 2 --strategy fsdp --steps 200 --warmup 20"
    run "rep $r N=4 DP xg_wt=$wt" "JDT_BACKEND=gloo JDT_XG_WT=$wt" "--gpus 4 --steps 200 --warmup 20"
  done
  for ov in 1 0; do
    run "rep $r DP2xPP2 LM overlap_sync=$ov" "JDT_BACKEND=gloo JDT_PP_OVERLAP_SYNC=$ov" \
      "--gpus 4 --strategy pp --dp 2 --model transformer --steps 60 --warmup 10"
  done
done
for r in 1 2; do
  run "rep $r headline (wt defaults)" "" "--steps 300 --warmup 30"
  run "rep $r 4-layer md_wt=1 (default)" "" "--num-layers 4 --steps 300 --warmup 30"
  run "rep $r 4-layer md_wt=3 (+ row-major shadow)" "JDT_MD_WT=3" "--num-layers 4 --steps 300 --warmup 30"
  run "rep $r pp8 md_wt=3" "JDT_MD_WT=3" "--strategy pp --hidden-layers 8 --steps 300 --warmup 30"
  run "rep $r pp8 md_wt=1" "JDT_MD_WT=1" "--strategy pp --hidden-layers 8 --steps 300 --warmup 30"
done
echo done
