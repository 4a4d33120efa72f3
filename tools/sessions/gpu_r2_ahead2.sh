#!/bin/bash
# Run-ahead on DP and FSDP (N = 1): GPU tests touching the fused engines, then the all-config table
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/ahead2
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu \
  -k "fsdp or run_ahead or fused or deterministic or checkpoint or entry" > gpurun_out/ahead2/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/ahead2/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/sessions/gpu_r2_allcfg.sh
