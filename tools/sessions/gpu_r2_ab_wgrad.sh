#!/bin/bash
# in-model A/B: weight-gradient GEMMs on a side stream (JDT_OVERLAP_WGRAD) on the transformer / GPipe MLP
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/abw
for rep in 1 2; do
for mode in "--model transformer --merge-microbatches" "--model transformer"; do
  for w in 0 1; do
    JDT_OVERLAP_WGRAD=$w timeout -k 10 200 python bench.py --strategy pp $mode --steps 300 --warmup 30 > gpurun_out/abw/b.log 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/abw/b.log; exit 1; }
    echo "rep $rep mode='$mode' wgrad_stream=$w: $(grep '^{' gpurun_out/abw/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
  done
done
done
