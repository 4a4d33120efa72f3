set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s21
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s21
T="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T "tests/test_grad_scale_gpu.py::test_xgmi_strategies_grad_scale" "tests/test_kernels_gpu.py::test_single_stage_pipeline_merge_gpu" "tests/test_xgmi_gpu.py::test_fsdp_persistent_exchange_matches_per_step_launches" "tests/test_xgmi_gpu.py::test_fsdp_over_xgmi_matches_single_device" "tests/test_xgmi_gpu.py::test_transformer_hybrid_over_xgmi_matches_single_device" "tests/test_kernels_gpu.py::test_xent_metric_slab_fold" tests/test_lm_gpu.py > $O/t1.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" $O/t1.log | tail -25; echo "tests rc=$rc"
