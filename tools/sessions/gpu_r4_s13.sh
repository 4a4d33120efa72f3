#!/bin/bash
# Round 4 session 13: A/B of the one-GPU run-ahead backward's phase-3 order -- its own
# (MFMA result straight into the epilogue, the pre-one-launch ISA, default) vs the N > 1
# kernel's (all MFMAs, then the epilogues; JDT_MLP2_P3S=1) -- alternating, 300 steps; then
# the run-ahead tests with both and the N = 2 one-launch step.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s13
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])'; }
for r in 1 2 3 4; do
  for p3 in 0 1; do
    JDT_MLP2_P3S=$p3 timeout -k 10 120 python bench.py --steps 300 --warmup 30 > gpurun_out/s13/b.log 2>&1 || { tail -5 gpurun_out/s13/b.log; exit 1; }
    echo "rep $r p3s=$p3: $(js gpurun_out/s13/b.log)"
  done
done
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_grad_scale_gpu.py -m gpu -q --timeout 120 \
  --timeout-method thread -k "ahead" > gpurun_out/s13/pytest.log 2>&1
rc=$?; echo "pytest run-ahead rc=$rc"; tail -2 gpurun_out/s13/pytest.log
[ $rc -ne 0 ] && exit $rc
JDT_BACKEND=gloo timeout -k 10 200 python bench.py --gpus 2 --steps 200 --warmup 20 > gpurun_out/s13/n2.log 2>&1 || { tail -5 gpurun_out/s13/n2.log; exit 1; }
echo "N=2 one-launch: $(js gpurun_out/s13/n2.log)"
echo done
