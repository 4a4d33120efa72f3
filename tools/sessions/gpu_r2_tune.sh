#!/bin/bash
# tuned GEMM table: GEMM + transformer GPU tests, shape table, transformer bench + profile,
# and the staged vs unstaged N=2 DP step under rocprofv3 (2 ranks sharing the GPU, one profiler per rank)
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/tune
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/tune/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/tune/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python tools/bench_gemm.py --groups 0 --json gpurun_out/tune/gemm.json > gpurun_out/tune/gemm.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --strategy pp --model transformer --merge-microbatches --steps 300 --warmup 30 > gpurun_out/tune/tf.log 2>&1; rc=$?
echo "tf rc=$rc"; grep '^{' gpurun_out/tune/tf.log | cut -c1-200; fatal $rc && exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tune/prof_tf -o tf -- python bench.py --strategy pp --model transformer --merge-microbatches --steps 60 --warmup 5 > gpurun_out/tune/prof_tf.log 2>&1
rc=$?; echo "prof tf rc=$rc"; fatal $rc && exit $rc
for st in 0 1; do
  for r in 0 1; do
    RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=2961$st JDT_BACKEND=gloo JDT_XGMI_STAGED=$st \
      timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tune/stg$st/r$r -o k -- \
      python bench.py --gpus 2 --steps 200 --warmup 20 --no-comm-sweep > gpurun_out/tune/stg${st}_r$r.log 2>&1 &
  done
  wait; echo "staged=$st done"; grep -h '^{' gpurun_out/tune/stg${st}_r0.log | cut -c1-160
done
