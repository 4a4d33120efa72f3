set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s17
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s17
# timing lab: JDT_MD_WT=17 reads the deep backward's AdamW state from one 1-KB window and
# never writes it back (wrong numbers, timing only): the price of the per-step state traffic
for rep in 1 2; do for wt in 1 17; do
  JDT_MD_WT=$wt timeout -k 10 200 python bench.py --num-layers 4 --steps 300 --warmup 30 > $O/d4.log 2>&1 || { tail -20 $O/d4.log; exit 3; }
  echo "deep4 wt=$wt: $(python -c "import json;d=json.loads(open('$O/d4.log').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
done; done
