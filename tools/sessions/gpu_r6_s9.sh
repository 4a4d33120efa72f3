set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s9
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s9
: > $O/ab.txt
for rep in 1 2 3; do for up in 1 0; do for w in 5 25; do
  JDT_GRAPH_UPLOAD=$up timeout -k 10 120 python bench.py --steps 20 --warmup $w > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 3; }
  echo "rep $rep upload $up warmup $w: $(python -c "import json;d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")" | tee -a $O/ab.txt
done; done; done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
tail -15 $O/pytest_gpu.log; echo "pytest rc=$rc"
