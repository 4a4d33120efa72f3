#!/bin/bash
# LM one-stage: microbatch count x stream count (4x4 default, 8x4, 8x8, 16x8)
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/mb8
for rep in 1 2; do
  for cfg in "4 4" "8 4" "8 8" "16 8" "16 16"; do
    set -- $cfg
    JDT_MB_STREAMS=$2 timeout -k 10 180 python bench.py --strategy pp --model transformer --microbatches $1 --steps 200 --warmup 20 > gpurun_out/mb8/b.log 2>&1 || { echo "bench $cfg failed"; tail -5 gpurun_out/mb8/b.log; exit 1; }
    echo "rep $rep mb=$1 streams=$2: $(grep '^{' gpurun_out/mb8/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["config"]["single_stage_mode"], j["config"]["num_microbatches"])')"
  done
done
