set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s5
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s5
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }   # test failures: go on; faults / timeouts: stop
timeout -k 10 900 $T "tests/test_xgmi_gpu.py::test_fsdp_persistent_exchange_matches_per_step_launches" tests/test_lm_gpu.py tests/test_bench_fallback_gpu.py > $O/t1.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/t1.log | tail -30; echo "tests rc=$rc"
ok $rc || exit $rc
for c in 0 2; do
  JDT_MB_STREAMS=1 JDT_WPASS_CFG=$c timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm_c$c.log 2>&1 || { tail -20 $O/lm_c$c.log; exit 3; }
  echo "lm layer-major wpass cfg $c: $(python -c "import json;d=json.loads(open('$O/lm_c$c.log').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['config']['single_stage_mode'])")"
done
timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm_default.log 2>&1 || { tail -20 $O/lm_default.log; exit 3; }
echo "lm default: $(python -c "import json;d=json.loads(open('$O/lm_default.log').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['config']['single_stage_mode'])")"
cd /tmp && JDT_MB_STREAMS=1 JDT_WPASS_CFG=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_lmlm -o lm -- python3 $GRAFT_REPO_ROOT/bench.py --strategy pp --model transformer --steps 50 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof_lmlm.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof_lmlm.log; exit 3; }
cd $GRAFT_REPO_ROOT
f=$(find $O/prof_lmlm -name '*kernel_trace.csv' | head -1); python tools/ktimeline.py $f --marker embed_fwd --steps 40 > $O/prof_lmlm.timeline.txt 2>&1; cat $O/prof_lmlm.timeline.txt | head -60
for k in 1 0; do
JDT_BACKEND=gloo JDT_FSDP_PST=$k timeout -k 10 300 python bench.py --gpus 2 --strategy fsdp --steps 200 --warmup 20 --autotune off --no-comm-sweep > $O/fsdp2_pst$k.log 2>&1 || { tail -20 $O/fsdp2_pst$k.log; exit 3; }
echo "fsdp2 pst=$k: $(tail -1 $O/fsdp2_pst$k.log | cut -c1-250)"
done
