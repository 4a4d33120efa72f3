#!/bin/bash
# Round 4: the GPU_MAX_HW_QUEUES=2 core dump of the 4-stream LM step, once, with the stream
# cap lifted (JDT_HWQ_CAP=0) and faulthandler on (bench.py), so a native crash prints the
# Python frame it happened under (stream creation, capture, instantiation or replay).
# Eager steps first (JDT_NO_GRAPH), then the captured step.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/hwq4
for mode in eager graph; do
  extra=""; [ $mode = eager ] && extra="--no-graph"
  GPU_MAX_HW_QUEUES=2 JDT_HWQ_CAP=0 JDT_MB_STREAMS=4 timeout -k 10 180 python -X faulthandler bench.py --steps 40 --warmup 5 \
    --strategy pp --model transformer $extra > gpurun_out/hwq4/$mode.log 2>&1
  rc=$?
  echo "hwq=2 streams=4 $mode rc=$rc"; tail -40 gpurun_out/hwq4/$mode.log
  [ $rc -ne 0 ] && exit $rc
done
echo done
