set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s28
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s28
T="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 600 $T tests/test_kernels_gpu.py -k "layernorm or lm" tests/test_lm_gpu.py > $O/t1.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" $O/t1.log | tail -15; echo "tests rc=$rc"
ok $rc || exit $rc
for sl in 0 1; do JDT_LN_SLAB=$sl timeout -k 10 120 python tools/bench_ln.py > $O/ln$sl.log 2>&1 || { tail -20 $O/ln$sl.log; exit 3; }; echo "slab=$sl: $(head -1 $O/ln$sl.log | grep -v amdgpu | cut -c1-230)"; grep ln_bwd $O/ln$sl.log | head -1 | cut -c1-230; done
for rep in 1 2 3; do for sl in 0 1; do
  JDT_LN_SLAB=$sl timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm.log 2>&1 || { tail -20 $O/lm.log; exit 3; }
  echo "lm slab=$sl: $(python -c "import json;d=json.loads(open('$O/lm.log').read().strip().splitlines()[-1]);print(d['ms_per_step'])")"
done; done
