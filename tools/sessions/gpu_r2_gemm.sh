#!/bin/bash
# GEMM sweep: single-GEMM configs and grouped-launch tiles on the transformer shapes (vs hipBLASLt)
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
for c in -1 11 12 14; do
  echo "=== cfg $c"; timeout -k 10 120 python tools/bench_gemm.py --cfg $c --json gpurun_out/gemm_cfg$c.json || exit $?
done
echo "=== groups"; timeout -k 10 120 python tools/bench_gemm.py --only "none" --groups 32,64,128 --json gpurun_out/gemm_groups.json || exit $?
timeout -k 10 300 python bench.py --strategy pp --model transformer --merge-microbatches --steps 100 --warmup 10 > gpurun_out/tf.log 2>&1; echo "tf rc=$?"; tail -1 gpurun_out/tf.log | cut -c1-300
