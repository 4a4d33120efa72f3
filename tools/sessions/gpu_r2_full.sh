#!/bin/bash
# full GPU validation: every GPU test, then smoke() and a default bench run
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/full
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full/pytest.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/full/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/full/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/full/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; grep '^{' gpurun_out/full/bench.log | cut -c1-200
