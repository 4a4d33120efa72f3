# AdamW constants pinned early in the one-step mlp2 / md kernels: deep + fused GPU tests, per-step
# headline (JDT_MLP2_PST=0), N = 2 shared one-launch DP / FSDP
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s33 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_grad_scale_gpu.py \
  -k "deep or fused or ahead or adam or mlp" > gpurun_out/r5s33/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r5s33/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r5s33/tests.log | head; exit 1; }
for rep in 1 2; do
  JDT_MLP2_PST=0 timeout -k 10 120 python bench.py --steps 300 --warmup 30 > gpurun_out/r5s33/p0.r$rep.log 2>&1 || exit 1
  echo "per-step launches (PST=0) 300 steps: $(grep -o '"value": [0-9.]*' gpurun_out/r5s33/p0.r$rep.log)"
done
export JDT_BACKEND=gloo
for st in "" "--strategy fsdp"; do
  timeout -k 10 300 python bench.py --gpus 2 --steps 200 --warmup 20 $st > gpurun_out/r5s33/n2.log 2>&1 || { tail -5 gpurun_out/r5s33/n2.log; exit 1; }
  echo "N=2 shared $st: $(grep -o '"value": [0-9.]*' gpurun_out/r5s33/n2.log)"
done
