set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s10
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s10
lm() {  # $1 label, rest env
  local lab=$1; shift
  env "$@" timeout -k 10 240 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > $O/lm.log 2>&1 || { tail -20 $O/lm.log; exit 3; }
  echo "$lab: $(python -c "import json;d=json.loads(open('$O/lm.log').read().strip().splitlines()[-1]);print(d['ms_per_step'])")" | tee -a $O/ab.txt
}
: > $O/ab.txt
for rep in 1 2; do
  lm "rep $rep default" JDT_NOP=1
  for wr in "16 1" "8 2" "8 1" "4 2" "4 1"; do set -- $wr; lm "rep $rep ln_bwd waves $1 rows $2" JDT_LN_WAVES=$1 JDT_LN_ROWS=$2; done
  for r in 1 2 8; do lm "rep $rep xent rpw $r" JDT_XENT_RPW=$r; done
done
T="python -u -m pytest -v --timeout 300 --timeout-method thread"; timeout -k 10 300 $T "tests/test_kernels_gpu.py::test_overlapped_adamw_equals_single_launch" > $O/t1.log 2>&1; rc=$?; grep -E "PASSED|FAILED|passed|failed" $O/t1.log | tail -4; echo "tests rc=$rc"
