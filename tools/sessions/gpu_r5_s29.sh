# returning logit atomics in the in-kernel GPipe stage and the loop kernel: their GPU tests
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s29 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_pp_chain_gpu.py \
  tests/test_xgmi_gpu.py tests/test_grad_scale_gpu.py tests/test_kernels_gpu.py -k "stage or chain or pipeline or loop or pp_" \
  > gpurun_out/r5s29/pp_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r5s29/pp_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r5s29/pp_tests.log | head; exit 1; }
