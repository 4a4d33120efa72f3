#!/bin/bash
# LayerNorm backward rows-per-wave sweep + transformer bench (merged microbatches)
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 120 python tools/bench_ln.py > gpurun_out/bench_ln.log 2>&1; rc=$?
echo "bench_ln rc=$rc"; cat gpurun_out/bench_ln.log | tail -5; fatal $rc && exit $rc
timeout -k 10 200 python bench.py --strategy pp --model transformer --merge-microbatches --steps 200 --warmup 20 > gpurun_out/bench_tf.log 2>&1; rc=$?
echo "tf rc=$rc"; grep '^{' gpurun_out/bench_tf.log | cut -c1-300
