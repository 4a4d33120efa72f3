#!/bin/bash
# in-model A/B of the vectorised GEMM epilogue (tile table off): transformer microbatch loop and merged
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/abe
for rep in 1 2; do
for mode in "" "--merge-microbatches"; do
  for e in 1 0; do
    JDT_GEMM_TUNE=0 JDT_GEMM_EPI_VEC=$e timeout -k 10 200 python bench.py --strategy pp --model transformer $mode --steps 300 --warmup 30 > gpurun_out/abe/b.log 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/abe/b.log; exit 1; }
    echo "rep $rep mode='$mode' epi_vec=$e: $(grep '^{' gpurun_out/abe/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
  done
done
done
