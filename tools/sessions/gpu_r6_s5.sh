set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s5
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s5
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_mlp2_persistent_gpu.py tests/test_smoke_gpu.py > $O/t1.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/t1.log | tail -20; echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
: > $O/ab.txt
for rep in 1 2 3; do
  for sync in barrier colblk; do
    JDT_MLP2_PST_SYNC=$sync timeout -k 10 120 python bench.py --steps 300 --warmup 30 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 3; }
    echo "rep $rep sync $sync steps300: $(python -c "import json;d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")" | tee -a $O/ab.txt
    JDT_MLP2_PST_SYNC=$sync timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 3; }
    echo "rep $rep sync $sync steps20: $(python -c "import json;d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")" | tee -a $O/ab.txt
  done
done
