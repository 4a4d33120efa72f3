set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s23
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s23
T="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 600 $T tests/test_kernels_gpu.py -k "layernorm or ln_ or attn or xent or lm" tests/test_lm_gpu.py > $O/t1.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" $O/t1.log | tail -25; echo "tests rc=$rc"
ok $rc || exit $rc
timeout -k 10 120 python tools/bench_ln.py > $O/ln.log 2>&1 || { tail -20 $O/ln.log; exit 3; }
head -2 $O/ln.log | grep -v amdgpu
for rep in 1 2 3; do for v in "JDT_LN_XCD=0 JDT_ATTN_XCD=0" "JDT_LN_XCD=1 JDT_ATTN_XCD=0" "JDT_LN_XCD=1"; do
  env $v timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm.log 2>&1 || { tail -20 $O/lm.log; exit 3; }
  echo "lm [$v]: $(python -c "import json;d=json.loads(open('$O/lm.log').read().strip().splitlines()[-1]);print(d['ms_per_step'])")"
done; done
