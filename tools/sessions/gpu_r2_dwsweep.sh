#!/bin/bash
# 512-row weight-gradient shapes: cfg x R x split-K sweep (isolated)
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/dw
: > gpurun_out/dw/sweep.txt
for c in 10 11 12 13; do for r in 1 2; do for sp in 1 2 4; do
  timeout -k 10 100 python tools/bench_gemm.py --cfg $c --r $r --splits $sp --only "fc1 dW 2k,qkv dW 2k,fc2 dW 2k,fc1 dX 2k,fc2 fwd 2k" > gpurun_out/dw/l.log 2>&1 || { echo "cfg $c r $r sp $sp rc=$?"; continue; }
  grep -E "dW 2k|dX 2k|fwd 2k" gpurun_out/dw/l.log | awk -v c=$c -v r=$r -v sp=$sp '{print "c"c" r"r" sp"sp": "$0}' >> gpurun_out/dw/sweep.txt
done; done; done
echo done
