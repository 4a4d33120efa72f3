set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s36
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s36
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_lm -o lm -- python3 $GRAFT_REPO_ROOT/bench.py --strategy pp --model transformer --steps 50 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof_lm.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof_lm.log; exit 3; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_head -o head -- python3 $GRAFT_REPO_ROOT/bench.py --steps 300 --warmup 30 > $GRAFT_REPO_ROOT/$O/prof_head.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof_head.log; exit 3; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_d4 -o d4 -- python3 $GRAFT_REPO_ROOT/bench.py --num-layers 4 --steps 200 --warmup 20 > $GRAFT_REPO_ROOT/$O/prof_d4.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof_d4.log; exit 3; }
cd $GRAFT_REPO_ROOT
f=$(find $O/prof_lm -name '*kernel_trace.csv' | head -1); python tools/ktimeline.py $f --marker embed_fwd --steps 40 > $O/prof_lm.timeline.txt 2>&1; head -24 $O/prof_lm.timeline.txt
head -4 $O/prof_head/head_kernel_stats.csv | cut -c1-200; head -7 $O/prof_d4/d4_kernel_stats.csv | cut -c1-200
