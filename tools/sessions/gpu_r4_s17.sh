#!/bin/bash
# Round 4 session 17: the driver form (20 steps, 5 warmup) by steps per graph (one 20-node graph
# vs several shorter replays: does the host's graph submission leave the GPU idle?), alternating.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s17
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); d=j["details"]; print(j["value"], j["ms_per_step"], d.get("steps_per_graph"))'; }
for r in 1 2 3; do
  for spg in 20 10 5 4 2 1; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --steps-per-graph $spg > gpurun_out/s17/d.log 2>&1 || { tail -5 gpurun_out/s17/d.log; exit 1; }
    echo "rep $r steps-per-graph $spg: $(js gpurun_out/s17/d.log)"
  done
done
echo done
