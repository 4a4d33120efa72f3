#!/bin/bash
# FSDP steps per graph 50 -> 200 (as DP): N = 1 2-layer / 4-layer, N = 2 shared 2-layer / 4-layer.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s41
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print(j["value"], j["ms_per_step"], c.get("step_launches", ""))'; }
for st in "--strategy fsdp" "--strategy fsdp --num-layers 4"; do
  for r in 1 2; do
    timeout -k 10 180 python bench.py --steps 300 --warmup 30 $st > gpurun_out/r5s41/n1.log 2>&1 || { tail -5 gpurun_out/r5s41/n1.log; exit 1; }
    echo "== N=1 $st: $(js gpurun_out/r5s41/n1.log)"
  done
done
for st in "--strategy fsdp" "--strategy fsdp --num-layers 4"; do
  JDT_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 200 --warmup 20 $st > gpurun_out/r5s41/n2.log 2>&1 || { tail -5 gpurun_out/r5s41/n2.log; exit 1; }
  echo "== N=2 shared $st: $(js gpurun_out/r5s41/n2.log)"
done
echo done
