# the one-launch DP / FSDP step at W = 4 and 8 (narrower models so the grids fit the shared GPU)
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s37 || exit 1
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_xgmi_gpu.py \
  -k "width6 or 256]" > gpurun_out/r5s37/tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed|\[dp ws" gpurun_out/r5s37/tests.log | tail -12; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r5s37/tests.log | head -20; exit 1; }
