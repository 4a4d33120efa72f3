set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/bench_all.jsonl
for a in "" "--num-layers 4" "--strategy fsdp" "--strategy fsdp --num-layers 4" "--strategy pp --hidden-layers 8" "--strategy pp --model transformer" "--accum fused" "--accum loop"; do
  timeout -k 10 180 python bench.py --steps 300 --warmup 30 $a > gpurun_out/b.log 2>&1 || { echo "bench $a failed"; tail -20 gpurun_out/b.log; exit 3; }
  echo "== $a"; tail -1 gpurun_out/b.log | cut -c1-220; tail -1 gpurun_out/b.log >> gpurun_out/bench_all.jsonl
done
