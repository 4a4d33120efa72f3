#!/bin/bash
# in-model A/B: vectorised-epilogue size threshold (outputs) on the transformer, loop and merged
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/abm
for mode in "" "--merge-microbatches"; do
  for th in 0 1048576 2097152 1000000000; do
    JDT_GEMM_EPI_MIN=$th timeout -k 10 200 python bench.py --strategy pp --model transformer $mode --steps 300 --warmup 30 > gpurun_out/abm/b.log 2>&1 || { echo "rc=$?"; tail -3 gpurun_out/abm/b.log; exit 1; }
    echo "mode='$mode' min=$th: $(grep '^{' gpurun_out/abm/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
  done
done
