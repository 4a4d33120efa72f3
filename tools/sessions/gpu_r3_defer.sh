#!/bin/bash
# Deferred weight-gradient W pass + vectorised AdamW epilogue: LM GPU tests, diagnostics, A/B benches
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/defer
timeout -k 10 300 python -u -m pytest tests/test_lm_gpu.py tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "lm or adamw or epilogue or transformer" > gpurun_out/defer/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/defer/pytest.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 200 python tools/diag_lm_epi_adamw.py --per-mb > gpurun_out/defer/diag_mb.log 2>&1; echo "diag rc=$?"; head -40 gpurun_out/defer/diag_mb.log
: > gpurun_out/defer/ab.jsonl
run() {  # label, env, args
  env $2 timeout -k 10 200 python bench.py --steps 200 --warmup 20 $3 > gpurun_out/defer/b.log 2>&1 || { echo "$1 failed"; tail -5 gpurun_out/defer/b.log; return 1; }
  echo "== $1: $(grep '^{' gpurun_out/defer/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
  grep '^{' gpurun_out/defer/b.log | sed "s/^{/{\"label\": \"$1\", /" >> gpurun_out/defer/ab.jsonl
}
LM="--strategy pp --model transformer"
run "lm layer-major epi-adamw" "JDT_LM_FUSED_OPT=1" "$LM" || exit 1
run "lm layer-major plain-adamw" "JDT_LM_FUSED_OPT=0" "$LM" || exit 1
run "lm per-mb defer epi-adamw" "JDT_DEFER_WGRAD=1 JDT_LM_FUSED_OPT=1" "$LM --microbatch-passes" || exit 1
run "lm per-mb defer plain-adamw" "JDT_DEFER_WGRAD=1 JDT_LM_FUSED_OPT=0" "$LM --microbatch-passes" || exit 1
run "lm per-mb no-defer epi-adamw" "JDT_DEFER_WGRAD=0 JDT_LM_FUSED_OPT=1" "$LM --microbatch-passes" || exit 1
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/defer/prof_mb -o run -- \
  python3 bench.py $LM --microbatch-passes --steps 100 --warmup 10 > gpurun_out/defer/prof.log 2>&1 || exit 1
