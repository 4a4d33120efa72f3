#!/bin/bash
# Layer-major LM with the deferred weight-gradient GEMMs on side streams (JDT_LM_WSTREAMS=k), per-microbatch passes
# on 4 streams with the W pass round-robin: GPU tests, alternating bench A/B
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/wp
timeout -k 10 300 python -u -m pytest tests/test_lm_gpu.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/wp/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|passed|failed|Error|rel diff|worst" gpurun_out/wp/pytest.log | tail -24
case $rc in 0) ;; *) exit $rc;; esac
for rep in 1 2; do
  for k in 1 2 3 4; do
    JDT_LM_WSTREAMS=$k timeout -k 10 180 python bench.py --strategy pp --model transformer --steps 200 --warmup 20 > gpurun_out/wp/b.log 2>&1 || { echo "bench k=$k failed"; tail -5 gpurun_out/wp/b.log; exit 1; }
    echo "rep $rep layer-major wstreams $k: $(grep '^{' gpurun_out/wp/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["config"]["single_stage_mode"])')"
  done
  timeout -k 10 180 python bench.py --strategy pp --model transformer --microbatch-passes --steps 200 --warmup 20 > gpurun_out/wp/b.log 2>&1 || { echo "bench mb failed"; tail -5 gpurun_out/wp/b.log; exit 1; }
  echo "rep $rep per-mb 4 streams + W pass round-robin: $(grep '^{' gpurun_out/wp/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["config"]["single_stage_mode"])')"
done
