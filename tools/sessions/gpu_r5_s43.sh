#!/bin/bash
# Steps per graph for the deep / pipeline replays (alternating, 3 reps, 300 steps): 4-layer DP at
# 50 / 25 / 10, GPipe-8 one stage at 50 / 20.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s43
v() { grep '^{' $1 | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])'; }
for r in 1 2 3; do
  line="rep $r 4-layer:"
  for s in 50 25 10; do
    timeout -k 10 180 python bench.py --steps 300 --warmup 30 --num-layers 4 --steps-per-graph $s > gpurun_out/r5s43/d$s.log 2>&1 || { tail -5 gpurun_out/r5s43/d$s.log; exit 1; }
    line="$line spg $s $(v gpurun_out/r5s43/d$s.log)"
  done
  echo "$line"
done
for r in 1 2; do
  line="rep $r pp8:"
  for s in 50 20; do
    timeout -k 10 180 python bench.py --steps 300 --warmup 30 --strategy pp --hidden-layers 8 --steps-per-graph $s > gpurun_out/r5s43/p$s.log 2>&1 || { tail -5 gpurun_out/r5s43/p$s.log; exit 1; }
    line="$line spg $s $(v gpurun_out/r5s43/p$s.log)"
  done
  echo "$line"
done
echo done
