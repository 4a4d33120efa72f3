#!/bin/bash
# Last check of the round: full GPU suite + smoke + driver-form bench on the final tree
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/last
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/last/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/last/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/last/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/last/smoke.log; exit 1; }
tail -1 gpurun_out/last/smoke.log
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/last/bench.log 2>&1 || { tail -5 gpurun_out/last/bench.log; exit 1; }
grep '^{' gpurun_out/last/bench.log
