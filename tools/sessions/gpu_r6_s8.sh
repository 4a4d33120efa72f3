set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s8
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s8
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
for rep in 1 2; do
  timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm.log 2>&1 || { tail -20 $O/lm.log; exit 3; }
  echo "rep $rep lm: $(python -c "import json;d=json.loads(open('$O/lm.log').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['config']['single_stage_mode'])")"
done
timeout -k 10 600 python tools/bench_lm_gemms.py --sweep 10,11,12,13,15,16,20,22,23,24,26,27 > $O/sweep.log 2> $O/sweep.err; rc=$?; cat $O/sweep.log; [ $rc -eq 0 ] || { tail -5 $O/sweep.err; exit $rc; }
timeout -k 10 300 python tools/bench_wpass.py --cfgs 2,4,5 > $O/wpass.log 2>&1; rc=$?; grep -v amdgpu.ids $O/wpass.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 $T tests/test_kernels_gpu.py -k "gemm or epilogue or adamw" tests/test_lm_gpu.py > $O/t1.log 2>&1; rc=$?
grep -E "passed|failed" $O/t1.log | tail -3; grep FAILED $O/t1.log | head; echo "tests rc=$rc"
for c in 1 2 3 4; do
  JDT_LN_GEMM_CFG=$c timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lmln.log 2>&1 || { tail -20 $O/lmln.log; exit 3; }
  echo "lm JDT_LN_GEMM_CFG=$c: $(python -c "import json;d=json.loads(open('$O/lmln.log').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['config']['single_stage_mode'])")"
done
