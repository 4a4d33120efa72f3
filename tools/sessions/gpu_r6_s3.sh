set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s3
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s3
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }   # test failures: go on; faults / timeouts: stop
timeout -k 10 900 $T "tests/test_xgmi_gpu.py::test_pipeline_stage_kernel_checkpoint_restore" tests/test_deterministic_gpu.py "tests/test_mlp2_persistent_gpu.py::test_persistent_run_ahead_deterministic_is_bitwise_equal" tests/test_ipc_pool_gpu.py tests/test_bench_fallback_gpu.py > $O/t1.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/t1.log | tail -30; echo "tests rc=$rc"
ok $rc || exit $rc
for k in 1 0; do
JDT_BACKEND=gloo JDT_DP_PST=$k timeout -k 10 300 python bench.py --gpus 2 --steps 200 --warmup 20 --autotune off --no-comm-sweep > $O/dp2_pst$k.log 2>&1 || { tail -20 $O/dp2_pst$k.log; exit 3; }
echo "dp2 pst=$k: $(tail -1 $O/dp2_pst$k.log | cut -c1-250)"
done
timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm_default.log 2>&1 || { tail -20 $O/lm_default.log; exit 3; }
echo "lm default: $(tail -1 $O/lm_default.log | cut -c1-300)"
JDT_MB_STREAMS=1 timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm_lm.log 2>&1 || { tail -20 $O/lm_lm.log; exit 3; }
echo "lm layer-major: $(tail -1 $O/lm_lm.log | cut -c1-300)"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_lm -o lm -- python3 $GRAFT_REPO_ROOT/bench.py --strategy pp --model transformer --steps 50 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof_lm.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof_lm.log; exit 3; }
cd /tmp && JDT_MB_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_lmlm -o lm -- python3 $GRAFT_REPO_ROOT/bench.py --strategy pp --model transformer --steps 50 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof_lmlm.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof_lmlm.log; exit 3; }
cd $GRAFT_REPO_ROOT
for d in prof_lm prof_lmlm; do f=$(find $O/$d -name '*kernel_trace.csv' | head -1); echo "== $d"; python tools/ktimeline.py $f --marker embed_fwd --steps 40 > $O/$d.timeline.txt 2>&1; cat $O/$d.timeline.txt; done
JDT_IPC_POOL=0 JDT_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29517 tools/xgmi_churn.py --iters 12 > $O/churn.log 2>&1; echo "churn rc=$?"; tail -2 $O/churn.log | cut -c1-400
