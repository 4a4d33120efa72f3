#!/bin/bash
# Whole GPU suite (no -x: every failure listed) + smoke, as the round-end driver runs them
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/suite
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/suite/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/suite/pytest.log | tail -12
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
