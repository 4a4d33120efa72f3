#!/bin/bash
# Round 3: S <= 128 attention kernels -- numerics, micro-bench A/B, in-model transformer step
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/attn
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attn128 or flash_attention or attention_fwd_bwd" -x -v --timeout 120 --timeout-method thread > gpurun_out/attn/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/attn/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/bench_attn.py > gpurun_out/attn/bench_attn.log 2>&1 || exit $?
cat gpurun_out/attn/bench_attn.log
for mode in "" "--microbatch-passes"; do
  for a in 1 0; do
    JDT_ATTN128=$a timeout -k 10 200 python bench.py --strategy pp --model transformer --steps 100 --warmup 10 $mode > gpurun_out/attn/b.log 2>&1 || exit $?
    echo "attn128=$a mode='$mode': $(grep '^{' gpurun_out/attn/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
  done
done
