set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s24
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s24
T="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 600 $T tests/test_lm_gpu.py tests/test_kernels_gpu.py -k "wpass or lm or embedding" > $O/t1.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" $O/t1.log | tail -15; echo "tests rc=$rc"
ok $rc || exit $rc
for rep in 1 2 3; do for pf in 0 1; do
  JDT_WPASS_PF=$pf timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm.log 2>&1 || { tail -20 $O/lm.log; exit 3; }
  echo "lm pf=$pf: $(python -c "import json;d=json.loads(open('$O/lm.log').read().strip().splitlines()[-1]);print(d['ms_per_step'])")"
done; done
