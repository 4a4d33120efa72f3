#!/bin/bash
# Round 4 session 16: the bench's one-launch fallback rehearsal (tests/test_bench_fallback_gpu.py),
# then the driver form (20 steps, 5 warmup) with the host's closing synchronize sleeping (default)
# vs spinning (JDT_SYNC_SPIN=1), alternating, and the 300-step form both ways.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s16
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; d=j["details"]; print(j["value"], j["ms_per_step"], d.get("host_sync"), c.get("one_launch_fallback", ""))'; }
timeout -k 10 600 python -u -m pytest tests/test_bench_fallback_gpu.py -v --timeout 500 --timeout-method thread \
  > gpurun_out/s16/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/s16/pytest.log | tail
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/s16/pytest.log | head -20; case $rc in 124|134|137|139) exit $rc;; esac; }
for r in 1 2 3 4; do
  for sp in 0 1; do
    timeout -k 10 120 env JDT_SYNC_SPIN=$sp python bench.py --steps 20 --warmup 5 > gpurun_out/s16/d.log 2>&1 || { tail -5 gpurun_out/s16/d.log; exit 1; }
    echo "driver form rep $r spin=$sp: $(js gpurun_out/s16/d.log)"
  done
done
for sp in 0 1; do
  timeout -k 10 180 env JDT_SYNC_SPIN=$sp python bench.py --steps 300 --warmup 30 > gpurun_out/s16/h.log 2>&1 || { tail -5 gpurun_out/s16/h.log; exit 1; }
  echo "300 steps spin=$sp: $(js gpurun_out/s16/h.log)"
done
echo done
