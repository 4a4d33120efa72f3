set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s41
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s41
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lm_gpu.py > $O/lm.log 2>&1 || { tail -30 $O/lm.log; exit 3; }
tail -1 $O/lm.log
for r in 1 2 3 4; do
  for c in 4 7; do
    JDT_WPASS_CFG=$c timeout -k 10 200 python bench.py --strategy pp --model transformer --steps 400 --warmup 40 > $O/b_${c}_${r}.log 2>&1 || { tail -20 $O/b_${c}_${r}.log; exit 3; }
    echo "wpass_cfg=$c run=$r $(grep -o '"ms_per_step": [0-9.]*' $O/b_${c}_${r}.log)"
  done
done
for c in 4 7; do
cd /tmp && JDT_WPASS_CFG=$c timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_$c -o lm -- python3 $GRAFT_REPO_ROOT/bench.py --strategy pp --model transformer --steps 50 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof_$c.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof_$c.log; exit 3; }
cd $GRAFT_REPO_ROOT; grep -E "wpass" $O/prof_$c/lm_kernel_stats.csv | cut -c1-150
done
