#!/bin/bash
# Final round-2 rocprofv3 kernel stats: 4-layer DP (layer-0 run-ahead) and the 1-GPU transformer step
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/fprof
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fprof/mlp4 -o run -- \
  python3 bench.py --num-layers 4 --steps 300 --warmup 30 > gpurun_out/fprof/mlp4.log 2>&1 || exit 1
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fprof/lm -o run -- \
  python3 bench.py --strategy pp --model transformer --steps 100 --warmup 10 > gpurun_out/fprof/lm.log 2>&1 || exit 1
find gpurun_out/fprof -name "*kernel_stats.csv"
