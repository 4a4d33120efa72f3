#!/bin/bash
# FSDP: replicated all-reduce folded into the reduce-scatter launch -- xGMI/FSDP tests + shared-GPU N=2/4 rehearsal
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/ff
timeout -k 10 600 python -u -m pytest tests/test_xgmi_gpu.py tests/test_grad_scale_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/ff/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/ff/pytest.log; [ $rc -ne 0 ] && exit $rc
export JDT_BACKEND=gloo
for n in 2 4; do for a in "--strategy fsdp" "--strategy fsdp --num-layers 4"; do
  timeout -k 10 240 python bench.py --gpus $n --steps 200 --warmup 20 $a > gpurun_out/ff/b.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/ff/b.log; exit 1; }
  echo "N=$n '$a': $(grep '^{' gpurun_out/ff/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["details"]["xgmi_selftest"])')"
done; done
