#!/bin/bash
# new-kernel tests first, then the full GPU suite, headline bench and both transformer modes
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/full
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "ln_gemm or attn128" -x -q --timeout 120 --timeout-method thread > gpurun_out/full/pytest_new.log 2>&1
rc=$?; echo "new rc=$rc"; tail -4 gpurun_out/full/pytest_new.log
[ $rc -ne 0 ] && exit $rc
for a in "--strategy pp --model transformer" "--strategy pp --model transformer --microbatch-passes"; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 $a > gpurun_out/full/b.log 2>&1 || { tail -5 gpurun_out/full/b.log; exit 1; }
  echo "'$a': $(grep '^{' gpurun_out/full/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/full/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/full/pytest_gpu.log
fatal $rc && exit $rc
timeout -k 10 200 python bench.py --steps 200 --warmup 20 > gpurun_out/full/b.log 2>&1 || { tail -5 gpurun_out/full/b.log; exit 1; }
echo "headline: $(grep '^{' gpurun_out/full/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
