#!/bin/bash
# final round-2 evidence: GEMM shape table vs hipBLASLt, transformer merged profile, headline profile
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/fin
timeout -k 10 150 python tools/bench_gemm.py --groups 0 --json gpurun_out/fin/gemm.json > gpurun_out/fin/gemm.log 2>&1 || exit $?
echo gemm done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin/prof_tf -o tf -- python bench.py --strategy pp --model transformer --merge-microbatches --steps 60 --warmup 5 > gpurun_out/fin/prof_tf.log 2>&1 || exit $?
echo tf prof done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin/prof_dp -o dp -- python bench.py --steps 400 --warmup 50 > gpurun_out/fin/prof_dp.log 2>&1 || exit $?
echo dp prof done
