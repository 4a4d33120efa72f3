#!/bin/bash
# Hardware queues per process (GPU_MAX_HW_QUEUES, box default 4) vs the concurrent-stream schedules
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/hwq
for rep in 1 2; do
  for q in 4 8 2; do
    for a in "--strategy pp --model transformer" "--accum loop --num-layers 4"; do
      GPU_MAX_HW_QUEUES=$q timeout -k 10 180 python bench.py --steps 200 --warmup 20 $a > gpurun_out/hwq/b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/hwq/b.log; exit 1; }
      echo "rep $rep hwq $q $a: $(grep '^{' gpurun_out/hwq/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
    done
  done
done
