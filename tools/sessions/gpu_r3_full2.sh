#!/bin/bash
# Full GPU suite + smoke after the concurrent microbatch-stream LM schedule, then the LM bench default vs layer-major
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/full2
timeout -k 10 800 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/full2/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|Error" gpurun_out/full2/pytest.log | tail -8
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full2/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/full2/smoke.log; exit 1; }
tail -1 gpurun_out/full2/smoke.log
for rep in 1 2; do
  for k in 4 1; do
    JDT_MB_STREAMS=$k timeout -k 10 180 python bench.py --strategy pp --model transformer --steps 300 --warmup 20 > gpurun_out/full2/b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/full2/b.log; exit 1; }
    echo "rep $rep JDT_MB_STREAMS=$k: $(grep '^{' gpurun_out/full2/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["config"]["single_stage_mode"])')"
    grep '^{' gpurun_out/full2/b.log >> gpurun_out/full2/lm.jsonl
  done
done
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/full2/prof -o run -- \
  python3 bench.py --strategy pp --model transformer --steps 100 --warmup 10 > gpurun_out/full2/prof.log 2>&1 || exit 1
echo prof ok
