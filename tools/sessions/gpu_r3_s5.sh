#!/bin/bash
# LM per-microbatch / layer-major A/B: round-3 tile table vs heuristic only (JDT_GEMM_TUNE=0),
# alternating; GEMM tests; deep-MLP phase stamps
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s5
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 150 --timeout-method thread -k "gemm" > gpurun_out/s5/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/s5/pytest.log | tail -4
case $rc in 0) ;; *) exit $rc;; esac
: > gpurun_out/s5/ab.jsonl
for rep in 1 2; do
  for tune in 1 0; do
    for a in "--strategy pp --model transformer --microbatch-passes" "--strategy pp --model transformer"; do
      JDT_GEMM_TUNE=$tune timeout -k 10 180 python bench.py --steps 200 --warmup 20 $a > gpurun_out/s5/b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/s5/b.log; exit 1; }
      echo "rep $rep tune=$tune $a: $(grep '^{' gpurun_out/s5/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
      grep '^{' gpurun_out/s5/b.log | sed "s/^{/{\"label\": \"rep $rep tune $tune\", /" >> gpurun_out/s5/ab.jsonl
    done
  done
done
timeout -k 10 120 python tools/stamp_deep.py --layers 4 > gpurun_out/s5/stamp_deep.log 2>&1 || { tail -5 gpurun_out/s5/stamp_deep.log; exit 1; }
grep -v amdgpu.ids gpurun_out/s5/stamp_deep.log
