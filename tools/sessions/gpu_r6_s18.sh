set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s18
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s18
T="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 600 $T tests/test_lm_gpu.py tests/test_kernels_gpu.py::test_xent_metric_slab_fold > $O/t1.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/t1.log | tail -25; echo "tests rc=$rc"
ok $rc || exit $rc
for rep in 1 2; do
  timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm.log 2>&1 || { tail -20 $O/lm.log; exit 3; }
  echo "lm: $(python -c "import json;d=json.loads(open('$O/lm.log').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['config']['single_stage_mode'])")"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_lm -o lm -- python3 $GRAFT_REPO_ROOT/bench.py --strategy pp --model transformer --steps 50 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof_lm.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof_lm.log; exit 3; }
cd $GRAFT_REPO_ROOT
f=$(find $O/prof_lm -name '*kernel_trace.csv' | head -1); python tools/ktimeline.py $f --marker embed_fwd --steps 40 > $O/prof_lm.timeline.txt 2>&1; head -30 $O/prof_lm.timeline.txt
