#!/bin/bash
# Round 4 final check on the final tree: the whole GPU suite, smoke(), the headline (300 steps and
# the driver form) and shared-GPU N = 2 DP / FSDP.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/final
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print(j["value"], j["ms_per_step"], c.get("step_launches", ""))'; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -2 gpurun_out/final/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/final/pytest_gpu.log | head -20; fatal $rc && exit $rc; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
for r in 1 2; do
  timeout -k 10 120 python bench.py --steps 300 --warmup 30 > gpurun_out/final/h.log 2>&1 || { tail -5 gpurun_out/final/h.log; exit 1; }
  echo "headline 300 steps: $(js gpurun_out/final/h.log)"
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/d.log 2>&1 || { tail -5 gpurun_out/final/d.log; exit 1; }
  echo "driver form: $(js gpurun_out/final/d.log)"
done
for a in "" "--strategy fsdp"; do
  timeout -k 10 200 env JDT_BACKEND=gloo python bench.py --gpus 2 --steps 200 --warmup 20 $a > gpurun_out/final/n.log 2>&1 || { echo "N=2 '$a' failed"; tail -5 gpurun_out/final/n.log; exit 1; }
  echo "N=2 $a: $(js gpurun_out/final/n.log)"
done
echo done
