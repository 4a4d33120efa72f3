#!/bin/bash
# Round 5 session 17: the whole GPU suite after the stage-kernel / FSDP-exchange / autotune
# changes, smoke(), the driver-form headline twice, and a rocprofv3 kernel-stats pass of it.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s17
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rs --durations=15 --timeout 300 --timeout-method thread \
  > gpurun_out/r5s17/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; grep -E "passed|failed|SKIP|FAILED|Error" gpurun_out/r5s17/pytest_gpu.log | tail -30
fatal $rc && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5s17/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/r5s17/smoke.log; exit 1; }
tail -2 gpurun_out/r5s17/smoke.log
for r in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/r5s17/d$r.log 2>&1 || { tail -5 gpurun_out/r5s17/d$r.log; exit 1; }
  grep '^{' gpurun_out/r5s17/d$r.log | cut -c1-300
done
timeout -k 10 120 python bench.py --steps 300 --warmup 30 > gpurun_out/r5s17/h300.log 2>&1 && grep '^{' gpurun_out/r5s17/h300.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5s17/prof -o headline -- python3 bench.py --steps 300 --warmup 30 \
  > gpurun_out/r5s17/prof.log 2>&1; rc=$?; echo "rocprof rc=$rc"
find gpurun_out/r5s17/prof -name "*kernel_stats.csv" | head -3
