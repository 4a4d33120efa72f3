#!/bin/bash
# headline DP: ordered partial logits (JDT_DETERMINISTIC=1) vs fp32 atomics; LN R=8 transformer check
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/det
for rep in 1 2 3; do for d in 0 1; do
  JDT_DETERMINISTIC=$d timeout -k 10 120 python bench.py --steps 500 --warmup 50 > gpurun_out/det/b.log 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/det/b.log; exit 1; }
  echo "rep $rep det=$d: $(grep '^{' gpurun_out/det/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
done; done
for d in 0 1; do
  JDT_DETERMINISTIC=$d timeout -k 10 120 python bench.py --num-layers 4 --steps 500 --warmup 50 > gpurun_out/det/b.log 2>&1 || exit 1
  echo "4-layer det=$d: $(grep '^{' gpurun_out/det/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
done
timeout -k 10 200 python bench.py --strategy pp --model transformer --merge-microbatches --steps 300 --warmup 30 > gpurun_out/det/t.log 2>&1 || exit 1
echo "tf merged: $(grep '^{' gpurun_out/det/t.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
