set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s4
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s4
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_mlp2_persistent_gpu.py "tests/test_xgmi_gpu.py::test_fsdp_persistent_exchange_matches_per_step_launches" tests/test_lm_gpu.py > $O/t1.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/t1.log | tail -30; echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/bench_wpass.py > $O/wpass.log 2>&1; rc=$?; tail -8 $O/wpass.log; [ $rc -eq 0 ] || exit $rc
for w in 1 0; do for mode in default lm; do
  E="JDT_MB_STREAMS=4"; [ $mode = lm ] && E="JDT_MB_STREAMS=1"
  env $E JDT_WPASS_ONE=$w timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm_${mode}_w$w.log 2>&1 || { tail -20 $O/lm_${mode}_w$w.log; exit 3; }
  echo "lm $mode wpass_one=$w: $(python -c "import json;d=json.loads(open('$O/lm_${mode}_w$w.log').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['config']['single_stage_mode'])")"
done; done
: > $O/ab.txt
for rep in 1 2; do for sync in barrier colblk; do
  JDT_MLP2_PST_SYNC=$sync timeout -k 10 120 python bench.py --steps 300 --warmup 30 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 3; }
  echo "rep $rep sync $sync steps300: $(python -c "import json;d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")" | tee -a $O/ab.txt
  JDT_MLP2_PST_SYNC=$sync timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 3; }
  echo "rep $rep sync $sync steps20: $(python -c "import json;d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")" | tee -a $O/ab.txt
done; done
: > $O/sweep.log
for c in -1 10 11 12 13 15 16 20 22 23 24 26 27; do
  echo "== cfg $c" >> $O/sweep.log
  timeout -k 10 120 python tools/bench_gemm.py --cfg $c --only "out fwd 2k,out dX 2k,qkv dX 2k,fc1 dX 2k,fc2 fwd 2k" >> $O/sweep.log 2>&1 || { echo "sweep cfg $c failed"; tail -5 $O/sweep.log; exit 3; }
done
grep -E "==|2k" $O/sweep.log | head -80
