#!/bin/bash
# Shared-GPU N = 2 kernel stats: DP vs FSDP (fused gather-once) steps, to see where FSDP2 loses to DP2
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 JDT_BACKEND=gloo && mkdir -p gpurun_out/s7
for s in dp fsdp; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s7/prof_$s -o run -- \
    python3 bench.py --gpus 2 --strategy $s --steps 200 --warmup 20 > gpurun_out/s7/$s.log 2>&1 || { tail -5 gpurun_out/s7/$s.log; exit 1; }
  grep '^{' gpurun_out/s7/$s.log | cut -c1-200
  for f in $(find gpurun_out/s7/prof_$s -name "*kernel_stats.csv"); do echo "== $f"; python tools/kstats.py $f 0 8 | cut -c1-150; done
done
