#!/bin/bash
# W pass GEMM tile under 4-stream concurrency: table (-1) vs forced bigger tiles
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/wcfg
for rep in 1 2; do
  for c in -1 11 12 14 20 22 23 24 26; do
    JDT_WPASS_CFG=$c timeout -k 10 180 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > gpurun_out/wcfg/b.log 2>&1 || { echo "bench cfg $c failed"; tail -3 gpurun_out/wcfg/b.log; continue; }
    echo "rep $rep wpass cfg $c: $(grep '^{' gpurun_out/wcfg/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
  done
done
