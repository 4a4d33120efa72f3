set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s2
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s2
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_smoke_gpu.py tests/test_mlp2_persistent_gpu.py "tests/test_xgmi_gpu.py::test_dp_persistent_exchange_matches_per_step_launches" "tests/test_xgmi_gpu.py::test_pipeline_stage_kernel_checkpoint_restore" > $O/t1.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|pst ws|passed|failed" $O/t1.log | tail -30; echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 $T tests/test_bench_fallback_gpu.py tests/test_xgmi_gpu.py -k "dp_over or bench or stage_kernel" > $O/t2.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/t2.log | tail -30; echo "tests2 rc=$rc"
[ $rc -eq 0 ] || exit $rc
for k in 1 0; do
JDT_BACKEND=gloo JDT_DP_PST=$k timeout -k 10 300 python bench.py --gpus 2 --steps 200 --warmup 20 --autotune off --no-comm-sweep > $O/dp2_pst$k.log 2>&1 || { tail -20 $O/dp2_pst$k.log; exit 3; }
echo "dp2 pst=$k: $(tail -1 $O/dp2_pst$k.log | cut -c1-200)"
done
timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm_default.log 2>&1 || { tail -20 $O/lm_default.log; exit 3; }
tail -1 $O/lm_default.log | cut -c1-300
JDT_MB_STREAMS=1 timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm_lm.log 2>&1 || { tail -20 $O/lm_lm.log; exit 3; }
tail -1 $O/lm_lm.log | cut -c1-300
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_lm -o lm -- python3 $GRAFT_REPO_ROOT/bench.py --strategy pp --model transformer --steps 50 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof_lm.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof_lm.log; exit 3; }
cd /tmp && JDT_MB_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_lmlm -o lm -- python3 $GRAFT_REPO_ROOT/bench.py --strategy pp --model transformer --steps 50 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof_lmlm.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof_lmlm.log; exit 3; }
cd $GRAFT_REPO_ROOT
for d in prof_lm prof_lmlm; do f=$(find $O/$d -name '*kernel_trace.csv' | head -1); echo "== $d"; python tools/ktimeline.py $f --marker embed_fwd --steps 40; done
