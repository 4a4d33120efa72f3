#!/bin/bash
# Round 4 session 8: the timed region without the torch record_function range (host ~20 us
# per replay): driver form x3 and 300 steps; the overlapped PP sync in 'auto' mode on the
# shared GPU (ranks_share_gpu -> one call) and forced on through the hybrid tests; a fresh
# rocprofv3 kernel-stats CSV of the headline and the 4-layer step with the write-through stores.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s8
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["config"].get("data_sync", ""))'; }
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/s8/d$r.log 2>&1 || { tail -5 gpurun_out/s8/d$r.log; exit 1; }
  echo "driver form $r: $(js gpurun_out/s8/d$r.log)"
done
timeout -k 10 120 python bench.py --steps 300 --warmup 30 > gpurun_out/s8/h.log 2>&1 || { tail -5 gpurun_out/s8/h.log; exit 1; }
echo "headline 300: $(js gpurun_out/s8/h.log)"
JDT_BACKEND=gloo timeout -k 10 200 python bench.py --gpus 4 --strategy pp --dp 2 --model transformer --steps 60 --warmup 10 \
  > gpurun_out/s8/lm.log 2>&1 || { tail -5 gpurun_out/s8/lm.log; exit 1; }
echo "DP2xPP2 LM auto: $(js gpurun_out/s8/lm.log)"
timeout -k 10 400 python -u -m pytest tests/test_xgmi_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "transformer_hybrid" > gpurun_out/s8/pytest_h.log 2>&1
rc=$?; echo "pytest hybrid rc=$rc"; tail -2 gpurun_out/s8/pytest_h.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/s8/pytest_h.log | head; exit $rc; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s8/prof_h -o run -- \
  python3 bench.py --steps 400 --warmup 50 > gpurun_out/s8/prof_h.log 2>&1 || { tail -5 gpurun_out/s8/prof_h.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s8/prof_4 -o run -- \
  python3 bench.py --num-layers 4 --steps 400 --warmup 50 > gpurun_out/s8/prof_4.log 2>&1 || { tail -5 gpurun_out/s8/prof_4.log; exit 1; }
find gpurun_out/s8 -name "*kernel_stats.csv" | head
echo done
