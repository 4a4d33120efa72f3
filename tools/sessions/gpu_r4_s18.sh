#!/bin/bash
# Round 4 session 18: HIP runtime knobs on the headline -- kernel arguments in device memory
# (HIP_FORCE_DEV_KERNARG) and pre-captured graph packets (DEBUG_CLR_GRAPH_PACKET_CAPTURE), each
# both ways against the default; driver form (20 steps) and 300 steps, plus the 4-layer step.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s18
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])'; }
for r in 1 2; do
  for e in "JDT_NOP=1" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"; do
    timeout -k 10 120 env $e python bench.py --steps 20 --warmup 5 > gpurun_out/s18/d.log 2>&1 || { echo "$e failed"; tail -5 gpurun_out/s18/d.log; exit 1; }
    a=$(js gpurun_out/s18/d.log)
    timeout -k 10 120 env $e python bench.py --steps 300 --warmup 30 > gpurun_out/s18/h.log 2>&1 || { echo "$e failed"; tail -5 gpurun_out/s18/h.log; exit 1; }
    b=$(js gpurun_out/s18/h.log)
    timeout -k 10 120 env $e python bench.py --steps 300 --warmup 30 --num-layers 4 > gpurun_out/s18/m.log 2>&1 || { echo "$e failed"; tail -5 gpurun_out/s18/m.log; exit 1; }
    c=$(js gpurun_out/s18/m.log)
    echo "rep $r $e: driver form $a | 300 steps $b | 4-layer $c"
  done
done
echo done
