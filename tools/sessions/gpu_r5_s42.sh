#!/bin/bash
# Steps per graph A/B (alternating, 3 reps): 4-layer DP at 50 vs 150 (300 steps); FSDP N = 2 shared
# 2-layer at 50 vs 200 (200 steps).
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s42
v() { grep '^{' $1 | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])'; }
for r in 1 2 3; do
  for s in 50 150; do
    timeout -k 10 180 python bench.py --steps 300 --warmup 30 --num-layers 4 --steps-per-graph $s > gpurun_out/r5s42/d$s.log 2>&1 || { tail -5 gpurun_out/r5s42/d$s.log; exit 1; }
  done
  echo "rep $r 4-layer: spg 50 $(v gpurun_out/r5s42/d50.log)  spg 150 $(v gpurun_out/r5s42/d150.log)"
done
for r in 1 2; do
  for s in 50 200; do
    JDT_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 200 --warmup 20 --strategy fsdp --steps-per-graph $s > gpurun_out/r5s42/f$s.log 2>&1 || { tail -5 gpurun_out/r5s42/f$s.log; exit 1; }
  done
  echo "rep $r fsdp N=2 shared: spg 50 $(v gpurun_out/r5s42/f50.log)  spg 200 $(v gpurun_out/r5s42/f200.log)"
done
echo done
