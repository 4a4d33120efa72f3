#!/bin/bash
# Per-microbatch LM passes on 1 / 2 / 4 streams: GPU tests (oracle + captured vs eager), alternating bench A/B
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/mbs
timeout -k 10 300 python -u -m pytest tests/test_lm_gpu.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/mbs/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|passed|failed|Error|rel diff|worst" gpurun_out/mbs/pytest.log | tail -20
case $rc in 0) ;; *) exit $rc;; esac
for rep in 1 2; do
  for k in 1 2 4; do
    JDT_MB_STREAMS=$k timeout -k 10 180 python bench.py --strategy pp --model transformer --microbatch-passes --steps 200 --warmup 20 > gpurun_out/mbs/b.log 2>&1 || { echo "bench k=$k failed"; tail -5 gpurun_out/mbs/b.log; exit 1; }
    echo "rep $rep streams $k: $(grep '^{' gpurun_out/mbs/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["config"]["single_stage_mode"])')"
  done
done
JDT_MB_STREAMS=2 timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mbs/prof -o run -- \
  python3 bench.py --strategy pp --model transformer --microbatch-passes --steps 100 --warmup 10 > gpurun_out/mbs/prof.log 2>&1 || exit 1
echo prof ok
