#!/bin/bash
# Round 5 session 6: sub-tick stamps of the in-kernel GPipe stage.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s6
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
export JDT_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 200 python tools/stamp_pp.py --gpus $n --microbatches 4 > gpurun_out/r5s6/stamp$n.log 2>&1; rc=$?
  grep -v -E "amdgpu.ids|Gloo|socket|connected peer" gpurun_out/r5s6/stamp$n.log | tail -14
  fatal $rc && exit $rc
done
exit 0
