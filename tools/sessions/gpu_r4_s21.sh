#!/bin/bash
# Round 4 session 21: exchange flags as global (not flat) accesses -- no flat instruction left in
# the fused kernels: the exchange / DP / FSDP xGMI tests, the grad-scale probes and the bench
# fallback, then shared-GPU N = 2 one-launch DP and FSDP (3 reps) and the 1-GPU headline.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s21
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print(j["value"], j["ms_per_step"], c.get("step_launches", ""))'; }
timeout -k 10 900 python -u -m pytest tests/test_xgmi_gpu.py tests/test_grad_scale_gpu.py tests/test_bench_fallback_gpu.py -m gpu -q \
  --timeout 300 --timeout-method thread > gpurun_out/s21/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/s21/pytest.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/s21/pytest.log | head -20; fatal $rc && exit $rc; exit 1; }
for r in 1 2 3; do
  for a in "" "--strategy fsdp"; do
    timeout -k 10 200 env JDT_BACKEND=gloo python bench.py --gpus 2 --steps 200 --warmup 20 $a > gpurun_out/s21/n.log 2>&1 || { echo "N=2 '$a' failed"; tail -5 gpurun_out/s21/n.log; exit 1; }
    echo "rep $r N=2 $a: $(js gpurun_out/s21/n.log)"
  done
  timeout -k 10 120 python bench.py --steps 300 --warmup 30 > gpurun_out/s21/h.log 2>&1 || { tail -5 gpurun_out/s21/h.log; exit 1; }
  echo "rep $r headline: $(js gpurun_out/s21/h.log)"
done
echo done
