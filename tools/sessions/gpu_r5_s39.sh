#!/bin/bash
# Kernel statistics of the 4-layer DP step and the GPipe-8 one-stage step (current kernels).
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s39
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5s39/deep4 -o run -- \
  python3 bench.py --steps 300 --warmup 30 --num-layers 4 > gpurun_out/r5s39/deep4.log 2>&1 || { tail -5 gpurun_out/r5s39/deep4.log; exit 1; }
grep '^{' gpurun_out/r5s39/deep4.log | cut -c1-100
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5s39/pp8 -o run -- \
  python3 bench.py --steps 300 --warmup 30 --strategy pp --hidden-layers 8 > gpurun_out/r5s39/pp8.log 2>&1 || { tail -5 gpurun_out/r5s39/pp8.log; exit 1; }
grep '^{' gpurun_out/r5s39/pp8.log | cut -c1-100
echo done
