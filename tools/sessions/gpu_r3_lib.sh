#!/bin/bash
# Plain bf16 GEMMs (no epilogue) on hipBLASLt (JDT_GEMM_LIB=1) vs the LDS-DMA kernels, LM step A/B
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/lib
JDT_GEMM_LIB=1 timeout -k 10 300 python -u -m pytest tests/test_lm_gpu.py -x -q -s --timeout 120 --timeout-method thread > gpurun_out/lib/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|Error|rel diff|worst" gpurun_out/lib/pytest.log | tail -12
case $rc in 0) ;; *) exit $rc;; esac
for rep in 1 2; do
  for lib in 0 1; do
    for k in 4 1; do
      JDT_GEMM_LIB=$lib JDT_MB_STREAMS=$k timeout -k 10 180 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > gpurun_out/lib/b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/lib/b.log; exit 1; }
      echo "rep $rep lib=$lib streams=$k: $(grep '^{' gpurun_out/lib/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["config"]["single_stage_mode"])')"
    done
  done
done
