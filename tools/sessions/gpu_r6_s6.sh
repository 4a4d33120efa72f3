set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s6
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s6
timeout -k 10 120 python tools/launch_floor.py > $O/floor.log 2>&1; rc=$?; cat $O/floor.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm_default.log 2>&1 || { tail -20 $O/lm_default.log; exit 3; }
echo "lm default: $(python -c "import json;d=json.loads(open('$O/lm_default.log').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['config']['single_stage_mode'])")"
timeout -k 10 300 python tools/bench_wpass.py > $O/wpass.log 2>&1; rc=$?; grep -v amdgpu.ids $O/wpass.log | tail -8; [ $rc -eq 0 ] || exit $rc
for c in 4 5; do
  JDT_WPASS_CFG=$c timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm_c$c.log 2>&1 || { tail -20 $O/lm_c$c.log; exit 3; }
  echo "lm wpass cfg $c: $(python -c "import json;d=json.loads(open('$O/lm_c$c.log').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['config']['single_stage_mode'])")"
done
