set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s16
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s16
T="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 600 $T tests/test_kernels_gpu.py -k "deep or run_ahead or fused_mlp" tests/test_grad_scale_gpu.py -k "run_ahead or deep or md" tests/test_deterministic_gpu.py > $O/t1.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/t1.log | tail -40; echo "tests rc=$rc"
ok $rc || exit $rc
for rep in 1 2; do for f in 0 1; do
  JDT_MD_FWD2=$f timeout -k 10 200 python bench.py --num-layers 4 --steps 300 --warmup 30 > $O/d4.log 2>&1 || { tail -20 $O/d4.log; exit 3; }
  echo "deep4 fwd2=$f: $(python -c "import json;d=json.loads(open('$O/d4.log').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
done; done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_d4 -o d4 -- python3 $GRAFT_REPO_ROOT/bench.py --num-layers 4 --steps 100 --warmup 20 > $GRAFT_REPO_ROOT/$O/prof_d4.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof_d4.log; exit 3; }
cd $GRAFT_REPO_ROOT; head -8 $O/prof_d4/d4_kernel_stats.csv | cut -c1-220
