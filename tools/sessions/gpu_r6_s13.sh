set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s13
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s13
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -3 $O/smoke.log
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 3; }
echo "headline: $(tail -1 $O/b.log | cut -c1-200)"
timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm.log 2>&1 || { tail -20 $O/lm.log; exit 3; }
echo "lm: $(python -c "import json;d=json.loads(open('$O/lm.log').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['config']['single_stage_mode'])")"
timeout -k 10 120 python tools/bench_attn.py > $O/attn.log 2>&1 || { tail -20 $O/attn.log; exit 3; }
cat $O/attn.log
timeout -k 10 120 python tools/bench_xent.py > $O/xent.log 2>&1 || { tail -20 $O/xent.log; exit 3; }
cat $O/xent.log | tail -20
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_lm -o lm -- python3 $GRAFT_REPO_ROOT/bench.py --strategy pp --model transformer --steps 50 --warmup 10 > $GRAFT_REPO_ROOT/$O/prof_lm.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof_lm.log; exit 3; }
cd $GRAFT_REPO_ROOT
f=$(find $O/prof_lm -name '*kernel_trace.csv' | head -1); python tools/ktimeline.py $f --marker embed_fwd --steps 40 > $O/prof_lm.timeline.txt 2>&1; head -40 $O/prof_lm.timeline.txt
