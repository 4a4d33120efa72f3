#!/bin/bash
# Early W pass (dedicated streams, per-part events) vs W pass after the join, LM default schedule
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/early
timeout -k 10 300 python -u -m pytest tests/test_lm_gpu.py -x -q -s --timeout 120 --timeout-method thread > gpurun_out/early/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|Error|rel diff|worst" gpurun_out/early/pytest.log | tail -14
case $rc in 0) ;; *) exit $rc;; esac
for rep in 1 2; do
  for e in 0 1 2 4; do
    JDT_WPASS_EARLY=$e timeout -k 10 180 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > gpurun_out/early/b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/early/b.log; exit 1; }
    echo "rep $rep early=$e: $(grep '^{' gpurun_out/early/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["config"]["single_stage_mode"])')"
  done
done
