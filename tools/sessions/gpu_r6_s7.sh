set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s7
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s7
: > $O/ab.txt
for rep in 1 2; do for wt in 0 1 2 3; do
  JDT_GEMM_WT=$wt timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm.log 2>&1 || { tail -20 $O/lm.log; exit 3; }
  echo "rep $rep JDT_GEMM_WT=$wt: $(python -c "import json;d=json.loads(open('$O/lm.log').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['config']['single_stage_mode'])")" | tee -a $O/ab.txt
done; done
for wt in 0 2; do
JDT_GEMM_WT=$wt timeout -k 10 300 python tools/bench_wpass.py --cfgs 2,4 > $O/wpass$wt.log 2>&1; rc=$?; echo "wpass WT=$wt"; grep -v amdgpu.ids $O/wpass$wt.log | tail -2; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python tools/bench_lm_gemms.py > $O/lmgemms.log 2>&1; rc=$?; grep -v amdgpu.ids $O/lmgemms.log; [ $rc -eq 0 ] || exit $rc
