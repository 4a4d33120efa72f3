set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6close4
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6close4
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" $O/pytest_gpu.log | tail -12; echo "pytest rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
grep "smoke ok" $O/smoke.log | cut -c1-160
: > $O/bench_all.jsonl
for a in "" "--optimizer sgd" "--num-layers 4" "--strategy fsdp" "--strategy fsdp --num-layers 4" "--strategy pp --hidden-layers 8" "--strategy pp --model transformer" "--accum loop"; do
  timeout -k 10 180 python bench.py --steps 300 --warmup 30 $a > $O/b.log 2>&1 || { echo "bench $a failed"; tail -20 $O/b.log; exit 3; }
  echo "== [$a] $(python -c "import json;d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"; tail -1 $O/b.log >> $O/bench_all.jsonl
done
for rep in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 3; }
  echo "driver form: $(python -c "import json;d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
done
