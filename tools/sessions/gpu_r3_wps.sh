#!/bin/bash
# LM default schedule: W pass round-robin over 1 / 2 / 3 / 4 of the microbatch streams
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/wps
for rep in 1 2; do
  for w in 4 1 2 3; do
    JDT_WPASS_STREAMS=$w timeout -k 10 180 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > gpurun_out/wps/b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/wps/b.log; exit 1; }
    echo "rep $rep wpass streams $w: $(grep '^{' gpurun_out/wps/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
  done
done
