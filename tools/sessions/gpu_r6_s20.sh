set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s20
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s20
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
tail -15 $O/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -2 $O/smoke.log
for rep in 1 2; do
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 3; }
echo "headline: $(tail -1 $O/b.log | cut -c1-260)"
done
