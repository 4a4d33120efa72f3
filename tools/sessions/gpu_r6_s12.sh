set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s12
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s12
T="python -u -m pytest -v --timeout 400 --timeout-method thread"
timeout -k 10 700 $T "tests/test_xgmi_gpu.py::test_pipeline_stage_kernel_equals_per_tick_launches" > $O/t1.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed" $O/t1.log | tail -12; echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for k in 1 0; do
  JDT_BACKEND=gloo JDT_PP_STAGE_SPARE=0 JDT_PP_KERNEL=$k timeout -k 10 400 python bench.py --gpus 8 --strategy pp --hidden-layers 8 --steps 200 --warmup 20 --autotune off > $O/pp8_k$k.log 2>&1 || { tail -20 $O/pp8_k$k.log; exit 3; }
  echo "pp8 kernel=$k: $(tail -1 $O/pp8_k$k.log | cut -c1-400)"
done
timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm.log 2>&1 || { tail -20 $O/lm.log; exit 3; }
echo "lm: $(python -c "import json;d=json.loads(open('$O/lm.log').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['config']['single_stage_mode'])")"
