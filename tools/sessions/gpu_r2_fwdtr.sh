#!/bin/bash
# mlp2_fwd LDS path (no W1^T copy: mode 0 / N > 1 / SGD) with transposing LDS reads: tests, then bench
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/fwdtr
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_grad_scale_gpu.py \
  -k "fused or mlp2 or mode or sgd or deterministic" > gpurun_out/fwdtr/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/fwdtr/pytest.log; [ $rc -ne 0 ] && exit $rc
val() { grep '^{' "$1" | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["details"]["final_loss"])'; }
for a in "--optimizer sgd" ""; do
  JDT_FUSED_OPT=0 timeout -k 10 120 python bench.py --steps 300 --warmup 30 $a > gpurun_out/fwdtr/b.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { tail -5 gpurun_out/fwdtr/b.log; exit $rc; }
  echo "mode0 '$a': $(val gpurun_out/fwdtr/b.log)"
done
JDT_BACKEND=gloo timeout -k 10 240 python bench.py --gpus 2 --steps 200 --warmup 20 > gpurun_out/fwdtr/b2.log 2>&1; rc=$?
[ $rc -ne 0 ] && { tail -5 gpurun_out/fwdtr/b2.log; exit $rc; }
echo "N=2 shared: $(val gpurun_out/fwdtr/b2.log)"
