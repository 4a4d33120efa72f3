#!/bin/bash
# Round 3: baseline profile of the transformer step, layer-major and per-microbatch passes.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/tprof
for mode in "" "--microbatch-passes"; do
  tag=$([ -z "$mode" ] && echo lm || echo mb)
  timeout -k 10 200 python bench.py --strategy pp --model transformer --steps 100 --warmup 10 $mode > gpurun_out/tprof/bench_$tag.log 2>&1 || exit $?
  grep '^{' gpurun_out/tprof/bench_$tag.log | cut -c1-400
  cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/tprof/$tag -o run -- \
    python3 /root/repo/bench.py --strategy pp --model transformer --steps 20 --warmup 3 $mode > /root/repo/gpurun_out/tprof/prof_$tag.log 2>&1 || exit $?
  cd /root/repo
done
