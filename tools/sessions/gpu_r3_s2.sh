#!/bin/bash
# FSDP loop fix + 32x32-MFMA GEMM tiles: targeted tests, the GEMM sweep with the new configs,
# the GPipe microbatch table (tools/pp_schedule.py), FSDP loop benches at N = 1 / 2 / 4
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s2
timeout -k 10 400 python -u -m pytest tests/test_grad_scale_gpu.py tests/test_kernels_gpu.py -q -x --timeout 150 --timeout-method thread -k "xgmi_strategies or mfma32" > gpurun_out/s2/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|Error" gpurun_out/s2/pytest.log | tail -8
case $rc in 0) ;; *) exit $rc;; esac
for c in -1 20 22 24 26 27; do
  timeout -k 10 120 python tools/bench_gemm.py --cfg $c > gpurun_out/s2/gemm_$c.log 2>&1 || { echo "gemm cfg $c failed"; tail -5 gpurun_out/s2/gemm_$c.log; exit 1; }
  echo "== cfg $c"; cat gpurun_out/s2/gemm_$c.log
done
timeout -k 10 400 python tools/pp_schedule.py --reps 100 --out gpurun_out/s2/pp_schedule.json > gpurun_out/s2/pp_schedule.log 2>&1 || { echo "pp_schedule failed"; tail -20 gpurun_out/s2/pp_schedule.log; exit 1; }
cat gpurun_out/s2/pp_schedule.log
: > gpurun_out/s2/fsdp.jsonl
timeout -k 10 120 python bench.py --steps 200 --warmup 20 --strategy fsdp --accum loop > gpurun_out/s2/b.log 2>&1 || { tail -5 gpurun_out/s2/b.log; exit 1; }
grep '^{' gpurun_out/s2/b.log | tee -a gpurun_out/s2/fsdp.jsonl | cut -c1-300
export JDT_BACKEND=gloo
for n in 2 4; do
  timeout -k 10 240 python bench.py --gpus $n --steps 100 --warmup 10 --strategy fsdp --accum loop > gpurun_out/s2/b.log 2>&1 || { tail -5 gpurun_out/s2/b.log; exit 1; }
  grep '^{' gpurun_out/s2/b.log | tee -a gpurun_out/s2/fsdp.jsonl | cut -c1-300
done
