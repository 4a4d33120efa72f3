#!/bin/bash
# Driver-form headline (--steps 20 --warmup 5) vs --warmup 25 (the 20-step graph replayed once before the timed region)
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/w20
for rep in 1 2 3; do
  for w in 5 25; do
    timeout -k 10 120 python bench.py --steps 20 --warmup $w > gpurun_out/w20/b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/w20/b.log; exit 1; }
    echo "rep $rep warmup $w: $(grep '^{' gpurun_out/w20/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["details"].get("p50_ms"))')"
  done
done
