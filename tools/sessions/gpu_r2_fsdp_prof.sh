#!/bin/bash
# N = 2 FSDP and GPipe, 2 ranks sharing the GPU, each rank under its own rocprofv3 (kernel list per step)
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/fp
for cfg in "fsdp:--strategy fsdp" "pp:--strategy pp --hidden-layers 8"; do
  name=${cfg%%:*}; args=${cfg#*:}
  for r in 0 1; do
    RANK=$r LOCAL_RANK=$r WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=29637 JDT_BACKEND=gloo \
      timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fp/$name/r$r -o k -- \
      python bench.py --gpus 2 --steps 200 --warmup 20 --no-comm-sweep $args > gpurun_out/fp/${name}_r$r.log 2>&1 &
  done
  wait; echo "$name done: $(grep -h '^{' gpurun_out/fp/${name}_r0.log | cut -c1-150)"
done
