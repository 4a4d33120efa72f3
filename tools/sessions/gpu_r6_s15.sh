set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s15
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s15
for rep in 1 2; do for opt in adamw sgd; do
  timeout -k 10 200 python bench.py --num-layers 4 --steps 300 --warmup 30 --optimizer $opt > $O/d4.log 2>&1 || { tail -20 $O/d4.log; exit 3; }
  echo "deep4 $opt: $(python -c "import json;d=json.loads(open('$O/d4.log').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
done; done
timeout -k 10 200 python tools/stamp_deep.py --layers 4 > $O/stamp_deep.log 2>&1 || { tail -20 $O/stamp_deep.log; exit 3; }
cat $O/stamp_deep.log
timeout -k 10 400 python tools/pp_schedule.py --reps 100 --counts 1,2,4 --out $O/pp_schedule.json > $O/pp_schedule.log 2>&1 || { tail -20 $O/pp_schedule.log; exit 3; }
tail -30 $O/pp_schedule.log
