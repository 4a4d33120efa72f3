set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s11
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s11
T="python -u -m pytest -v --timeout 400 --timeout-method thread"
timeout -k 10 600 $T "tests/test_grad_scale_gpu.py::test_pipeline_stage_kernel_adam_scale" > $O/t1.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed|Error" $O/t1.log | tail -12; echo "tests rc=$rc"
