set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s4
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s4
timeout -k 10 300 python tools/bench_wpass.py > $O/wpass.log 2>&1; rc=$?; cat $O/wpass.log | tail -12; [ $rc -eq 0 ] || exit $rc
: > $O/sweep.log
for c in -1 10 11 12 13 14 15 16 20 21 22 23 24 25 26 27; do
  echo "== cfg $c" >> $O/sweep.log
  timeout -k 10 120 python tools/bench_gemm.py --cfg $c --only "out fwd 2k,out dX 2k,qkv dX 2k,fc1 dX 2k,fc2 fwd 2k" >> $O/sweep.log 2>&1 || { echo "sweep cfg $c failed"; tail -5 $O/sweep.log; exit 3; }
done
grep -E "==|2k" $O/sweep.log | head -120
T="python -u -m pytest -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_lm_gpu.py > $O/t_lm.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/t_lm.log | tail -20; echo "lm tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for w in 1 0; do
for mode in default lm; do
  E=""; [ $mode = lm ] && E="JDT_MB_STREAMS=1"
  env $E JDT_WPASS_ONE=$w timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm_${mode}_w$w.log 2>&1 || { tail -20 $O/lm_${mode}_w$w.log; exit 3; }
  echo "lm $mode wpass_one=$w: $(tail -1 $O/lm_${mode}_w$w.log | cut -c180-260)"
done; done
cd /tmp && JDT_MB_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_lmlm -o lm -- python3 $GRAFT_REPO_ROOT/bench.py --strategy pp --model transformer --steps 50 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof_lmlm.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof_lmlm.log; exit 3; }
cd $GRAFT_REPO_ROOT; f=$(find $O/prof_lmlm -name '*kernel_trace.csv' | head -1); python tools/ktimeline.py $f --marker embed_fwd --steps 40 > $O/prof_lmlm.timeline.txt 2>&1; cat $O/prof_lmlm.timeline.txt | head -30
