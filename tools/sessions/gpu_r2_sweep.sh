#!/bin/bash
# tile sweep after the vectorised epilogue: every shape at cfg 10..14 (no split forcing), grouped tiles
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/sw
for c in 10 11 12 13 14; do
  timeout -k 10 150 python tools/bench_gemm.py --cfg $c --json gpurun_out/sw/cfg$c.json > gpurun_out/sw/cfg$c.log 2>&1 || { echo "cfg $c rc=$?"; exit 1; }
  echo "cfg $c done"
done
timeout -k 10 150 python tools/bench_gemm.py --only none --groups 32,64,128,0 --json gpurun_out/sw/groups.json > gpurun_out/sw/groups.log 2>&1; echo "groups rc=$?"
