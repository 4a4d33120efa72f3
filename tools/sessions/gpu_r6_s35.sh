set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s35
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s35
T="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 600 $T tests/test_kernels_gpu.py -k "layernorm or lm or pipeline" tests/test_lm_gpu.py > $O/t1.log 2>&1; rc=$?
grep -E "FAIL|Error|passed|failed" $O/t1.log | tail -15; echo "tests rc=$rc"
ok $rc || exit $rc
for rep in 1 2 3; do for v in 0 1; do
  JDT_LN_DEFER=$v timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm.log 2>&1 || { tail -20 $O/lm.log; exit 3; }
  echo "lm defer=$v: $(python -c "import json;d=json.loads(open('$O/lm.log').read().strip().splitlines()[-1]);print(d['ms_per_step'])")"
done; done
