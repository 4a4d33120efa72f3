#!/bin/bash
# GEMM (cfg, split-K) sweep on the shapes still below hipBLASLt (profiles/r3_gemm_mfma32_sweep.txt)
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s4
ONLY="fc1 fwd,fc2 fwd,head fwd,fc1 dX,fc2 dX,fc2 fwd 2k,fc1 dW 2k,fc1 fwd 2k,fc2 dX 2k,fc1 dX 2k"
for c in 10 11 12 13 20 21 22 23 26; do
  for sp in 1 2 4; do
    timeout -k 10 120 python tools/bench_gemm.py --cfg $c --splits $sp --only "$ONLY" > gpurun_out/s4/g.log 2>&1 || { echo "cfg $c sp $sp failed"; tail -3 gpurun_out/s4/g.log; continue; }
    grep -v amdgpu.ids gpurun_out/s4/g.log | grep -v "^shape" | sed "s/^/cfg $c sp $sp | /"
  done
done
