set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s1
timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm_default.log 2>&1 || { tail -20 $O/lm_default.log; exit 3; }
tail -1 $O/lm_default.log | cut -c1-400
JDT_MB_STREAMS=1 timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm_lm.log 2>&1 || { tail -20 $O/lm_lm.log; exit 3; }
tail -1 $O/lm_lm.log | cut -c1-400
timeout -k 10 300 python tools/bench_gemm.py --json $O/gemm.json > $O/gemm.log 2>&1 || { tail -20 $O/gemm.log; exit 3; }
cat $O/gemm.log
cd /tmp && JDT_MB_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_lm -o lm -- python3 $GRAFT_REPO_ROOT/bench.py --strategy pp --model transformer --steps 50 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof_lm.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof_lm.log; exit 3; }
cd $GRAFT_REPO_ROOT; f=$(find $O/prof_lm -name '*kernel_stats.csv' | head -1); python tools/kstats.py $f 60 30
