#!/bin/bash
# 8-wave / 128-tile configs with split-K on the long-K 2048-token shapes (not in the earlier sweeps)
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/gsweep
SH="fc2 fwd 2k,fc1 dX 2k,fc2 dW 2k,qkv dW 2k,fc1 dW 2k"
timeout -k 10 120 python tools/bench_gemm.py --only "$SH" > gpurun_out/gsweep/base.txt 2>&1 || exit 1
echo "== table"; grep -E "2k" gpurun_out/gsweep/base.txt | head -8
for cfg in 14 15 16 17 18; do
  for sp in 1 2 4; do
    timeout -k 10 120 python tools/bench_gemm.py --only "$SH" --cfg $cfg --splits $sp > gpurun_out/gsweep/c${cfg}_s${sp}.txt 2>&1 || { echo "cfg $cfg sp $sp failed"; tail -3 gpurun_out/gsweep/c${cfg}_s${sp}.txt; continue; }
    echo "== cfg $cfg splits $sp"; grep -E "2k" gpurun_out/gsweep/c${cfg}_s${sp}.txt | head -8
  done
done
