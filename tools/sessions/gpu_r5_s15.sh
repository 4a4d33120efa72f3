#!/bin/bash
# Round 5 session 15: end-of-step stamps of the GPipe stage kernel.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 JDT_BACKEND=gloo && mkdir -p gpurun_out/r5s15
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
for n in 2 4; do
  timeout -k 10 200 python tools/stamp_pp.py --gpus $n --microbatches 2 > gpurun_out/r5s15/stamp$n.log 2>&1; rc=$?
  grep -v -E "amdgpu.ids|Gloo|socket|connected peer" gpurun_out/r5s15/stamp$n.log | tail -16
  fatal $rc && exit $rc
done
exit 0
