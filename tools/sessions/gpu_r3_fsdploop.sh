#!/bin/bash
# FSDP fused per-minibatch loop + one-row epilogue units: tests, then A/B benches
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/fl
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_lm_gpu.py tests/test_grad_scale_gpu.py -q -x --timeout 150 --timeout-method thread -k "fsdp or lm or epilogue or gemm or xgmi_strategies" > gpurun_out/fl/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/fl/pytest.log; grep "fsdp loop\|apart" gpurun_out/fl/pytest.log | head -20
case $rc in 124|134|137|139) exit $rc;; esac
: > gpurun_out/fl/ab.jsonl
run() {  # label, env, args
  env $2 timeout -k 10 240 python bench.py --steps 200 --warmup 20 $3 > gpurun_out/fl/b.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/fl/b.log; return 1; }
  echo "== $1: $(grep '^{' gpurun_out/fl/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["config"].get("gather_once"))')"
  grep '^{' gpurun_out/fl/b.log | sed "s/^{/{\"label\": \"$1\", /" >> gpurun_out/fl/ab.jsonl
}
LM="--strategy pp --model transformer"
run "lm layer-major epi-adamw" "JDT_LM_FUSED_OPT=1" "$LM" || exit 1
run "lm layer-major plain-adamw" "JDT_LM_FUSED_OPT=0" "$LM" || exit 1
run "lm per-mb defer epi-adamw" "JDT_LM_FUSED_OPT=1" "$LM --microbatch-passes" || exit 1
run "lm per-mb defer plain-adamw" "JDT_LM_FUSED_OPT=0" "$LM --microbatch-passes" || exit 1
run "fsdp loop fused" "JDT_X=1" "--strategy fsdp --accum loop" || exit 1
run "fsdp loop fused L4" "JDT_X=1" "--strategy fsdp --accum loop --num-layers 4" || exit 1
export JDT_BACKEND=gloo
for n in 2 4; do
  run "fsdp$n loop fused" "JDT_X=1" "--gpus $n --strategy fsdp --accum loop" || exit 1
  run "fsdp$n kernel" "JDT_X=1" "--gpus $n --strategy fsdp" || exit 1
  run "dp$n kernel" "JDT_X=1" "--gpus $n" || exit 1
done
