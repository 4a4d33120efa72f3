#!/bin/bash
# in-model A/B of the GEMM tile table: transformer merged / microbatch loop, hybrid-shape, x tune on/off
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/abt
for rep in 1 2; do
for mode in "--merge-microbatches" ""; do
  for t in 1 0; do
    JDT_GEMM_TUNE=$t timeout -k 10 200 python bench.py --strategy pp --model transformer $mode --steps 300 --warmup 30 > gpurun_out/abt/b.log 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/abt/b.log; exit 1; }
    echo "rep $rep mode='$mode' tune=$t: $(grep '^{' gpurun_out/abt/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
  done
done
done
