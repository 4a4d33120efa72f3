#!/bin/bash
# Round 5 session 18: rocprofv3 kernel statistics (csv) of the headline step and of the
# one-stage transformer LM step (BASELINE config #5 on one GPU).
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s18
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r5s18/head -o head -- python3 bench.py --steps 300 --warmup 30 \
  > gpurun_out/r5s18/head.log 2>&1; echo "head rc=$?"
timeout -k 10 300 python bench.py --strategy pp --model transformer --steps 100 --warmup 10 > gpurun_out/r5s18/lm.log 2>&1; echo "lm rc=$?"
grep '^{' gpurun_out/r5s18/lm.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r5s18/lm -o lm -- python3 bench.py --strategy pp --model transformer --steps 100 --warmup 10 \
  > gpurun_out/r5s18/lmprof.log 2>&1; echo "lm prof rc=$?"
find gpurun_out/r5s18 -name "*stats*.csv"
