#!/bin/bash
# driver-style short bench (--steps 20 --warmup 5): steps per hipGraph 20 / 10 / 5 / 4 / 2
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/spg
for rep in 1 2 3; do for spg in 20 10 5 4 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --steps-per-graph $spg > gpurun_out/spg/b.log 2>&1 || { echo "rc=$?"; exit 1; }
  echo "rep $rep spg=$spg: $(grep '^{' gpurun_out/spg/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
done; done
