#!/bin/bash
# AHEAD_MB 20-step dropout-stream test, LN-GEMM tile sweep, per-mb / layer-major LM profiles
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s6
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_lm_gpu.py -q -x --timeout 150 --timeout-method thread -k "mb_streams or deep_run_ahead or adamw_and_step or epilogue_adamw or lm or set_batch" > gpurun_out/s6/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|Error|displacement" gpurun_out/s6/pytest.log | tail -8
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 200 python tools/bench_ln_gemm.py > gpurun_out/s6/ln_gemm.log 2>&1 || { tail -5 gpurun_out/s6/ln_gemm.log; exit 1; }
grep -v amdgpu.ids gpurun_out/s6/ln_gemm.log
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s6/prof_lmmb -o run -- \
  python3 bench.py --strategy pp --model transformer --microbatch-passes --steps 100 --warmup 10 > gpurun_out/s6/prof.log 2>&1 || exit 1
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s6/prof_lm -o run -- \
  python3 bench.py --strategy pp --model transformer --steps 100 --warmup 10 > gpurun_out/s6/prof2.log 2>&1 || exit 1
python tools/kstats.py gpurun_out/s6/prof_lmmb/run_kernel_stats.csv 160 14 | cut -c1-150
