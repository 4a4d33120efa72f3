set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 150 --timeout-method thread -k "p2p or pipeline" > gpurun_out/pytest_pp.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_pp.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
for a in "--strategy pp --hidden-layers 8" "--strategy pp --model transformer"; do
  timeout -k 10 180 python bench.py --steps 300 --warmup 30 $a > gpurun_out/b.log 2>&1 || { echo "bench $a failed"; tail -20 gpurun_out/b.log; exit 3; }
  echo "== $a"; tail -1 gpurun_out/b.log
done
