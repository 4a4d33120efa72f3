# A/B of the XCD-contiguous backward tile map (JDT_XCD_TILES=1, default) against the
# identity map (0) on the fused MLP steps, 1 GPU, alternating runs.
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mlp2 or deep or md_ or fused" > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 3; }
tail -2 gpurun_out/ab_tests.log
: > gpurun_out/ab_xcd.jsonl
for rep in 1 2; do
  for x in ${XS:-0 1}; do
    for a in "" "--num-layers 4"; do
      JDT_XCD_TILES=$x timeout -k 10 120 python bench.py --steps 2000 --warmup 100 $a > gpurun_out/ab.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/ab.log; exit 3; }
      v=$(grep '^{' gpurun_out/ab.log | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')
      echo "xcd=$x rep=$rep [$a] $v" | tee -a gpurun_out/ab_xcd.jsonl
    done
  done
done
