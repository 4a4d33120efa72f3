set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s29
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s29
T="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
for r in 1 2 4; do
JDT_LN_FWD_ROWS=$r timeout -k 10 300 $T tests/test_kernels_gpu.py -k "layernorm or ln_gemm" > $O/t$r.log 2>&1; rc=$?
echo "rows $r: $(grep -E "passed|failed" $O/t$r.log | tail -1)"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
for rep in 1 2 3; do for r in 1 2 4; do
  JDT_LN_FWD_ROWS=$r timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm.log 2>&1 || { tail -20 $O/lm.log; exit 3; }
  echo "lm rows=$r: $(python -c "import json;d=json.loads(open('$O/lm.log').read().strip().splitlines()[-1]);print(d['ms_per_step'])")"
done; done
