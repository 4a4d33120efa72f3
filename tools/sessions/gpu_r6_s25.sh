set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s25
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s25
for rep in 1 2; do for c in 4 0 1 2 3 5; do
  JDT_WPASS_CFG=$c timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm.log 2>&1 || { tail -20 $O/lm.log; exit 3; }
  echo "lm wpass cfg $c: $(python -c "import json;d=json.loads(open('$O/lm.log').read().strip().splitlines()[-1]);print(d['ms_per_step'])")"
done; done
