#!/bin/bash
# The driver's bench contract after the last bench.py edit: default run + deep configs' JSON details
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/bc
for a in "--steps 20 --warmup 5" "--num-layers 4 --steps 100 --warmup 10" "--strategy fsdp --num-layers 4 --steps 100 --warmup 10"; do
  timeout -k 10 120 python bench.py $a > gpurun_out/bc/b.log 2>&1 || { tail -5 gpurun_out/bc/b.log; exit 1; }
  grep '^{' gpurun_out/bc/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["steps"], j["warmup"], j["config"].get("step_launches"), j["details"]["hipgraph"], j["details"]["steps_per_graph"])'
done
