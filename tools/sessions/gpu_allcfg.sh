set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
: > gpurun_out/bench_all.jsonl
for a in "" "--num-layers 4" "--num-layers 3" "--strategy fsdp" "--strategy fsdp --num-layers 4" "--strategy pp --hidden-layers 8" "--strategy pp --model transformer" "--strategy pp --model transformer --merge-microbatches" "--accum fused" "--accum loop" "--accum scan"; do
  timeout -k 10 180 python bench.py --steps 300 --warmup 30 $a > gpurun_out/b.log 2>&1 || { echo "bench $a failed"; tail -20 gpurun_out/b.log; exit 3; }
  echo "== $a"; tail -1 gpurun_out/b.log | cut -c1-200; tail -1 gpurun_out/b.log >> gpurun_out/bench_all.jsonl
done
bash tools/sessions/gpu_multiproc_bench.sh
