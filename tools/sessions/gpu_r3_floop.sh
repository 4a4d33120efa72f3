#!/bin/bash
# FSDP per-minibatch loop at N = 1 on 2 streams (4 layers): GPU tests + alternating bench A/B
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/floop
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -s --timeout 120 --timeout-method thread -k "fsdp" > gpurun_out/floop/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|Error" gpurun_out/floop/pytest.log | tail -6
case $rc in 0) ;; *) exit $rc;; esac
for rep in 1 2; do
  for k in 1 0; do
    JDT_LOOP_STREAMS=$k timeout -k 10 180 python bench.py --strategy fsdp --accum loop --num-layers 4 --steps 300 --warmup 20 > gpurun_out/floop/b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/floop/b.log; exit 1; }
    echo "rep $rep fsdp loop 4-layer JDT_LOOP_STREAMS=$k: $(grep '^{' gpurun_out/floop/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
  done
done
