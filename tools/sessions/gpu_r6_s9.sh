set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s9
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s9
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?
tail -15 $O/pytest_gpu.log; echo "pytest rc=$rc"
