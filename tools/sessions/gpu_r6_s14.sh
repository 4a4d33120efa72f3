set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s14
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s14
T="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }   # test failures: go on; faults / timeouts: stop
timeout -k 10 600 $T tests/test_kernels_gpu.py -k "xent" tests/test_lm_gpu.py > $O/t1.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/t1.log | tail -40; echo "tests rc=$rc"
ok $rc || exit $rc
for rep in 1 2; do
for v in "JDT_XENT_SLAB=0 JDT_LM_RANGES_SIDE=0" "JDT_LM_RANGES_SIDE=0" "JDT_XENT_SLAB=0" "JDT_XENT_SLAB=1"; do
  env $v timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm.log 2>&1 || { tail -20 $O/lm.log; exit 3; }
  echo "lm [$v]: $(python -c "import json;d=json.loads(open('$O/lm.log').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['config']['single_stage_mode'])")"
done; done
cd /tmp
for m in warm cold; do
  fl=""; [ $m = cold ] && fl="--cold"
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_$m -o p -- python3 $GRAFT_REPO_ROOT/tools/pmc_lm_gemm.py $fl > $GRAFT_REPO_ROOT/$O/pmc_$m.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/pmc_$m.log; exit 3; }
done
cd $GRAFT_REPO_ROOT
for m in warm cold; do f=$(find $O/pmc_$m -name '*counter_collection.csv' | head -1); echo "== $m"; python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    if "gemm" in r.get("Kernel_Name", ""):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    v = v[5:]
    print(k, "median", sorted(v)[len(v) // 2], "n", len(v))
PY
done
