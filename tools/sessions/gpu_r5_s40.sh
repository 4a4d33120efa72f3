#!/bin/bash
# Driver form (--steps 20 --warmup 5) A/B: the timed region is the 20-step graph's FIRST launch.
# A = default, B = JDT_GRAPH_UPLOAD=1 (hipGraphUpload after capture), C = --warmup 25 (the timed
# launch is that graph's second).  Alternating, 3 reps.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s40
timeout -k 10 60 python -c "
import torch
from jax_distributed_tuts_amd.parallel.fused_mlp import upload_graphs
x = torch.zeros(16, device='cuda'); g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g): x.add_(1)
print('upload ok', upload_graphs([g])); g.replay(); torch.cuda.synchronize(); print(x[0].item())
" 2>&1 | grep -v amdgpu.ids || exit 1
v() { grep '^{' $1 | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])'; }
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/r5s40/a$r.log 2>&1 || { tail -5 gpurun_out/r5s40/a$r.log; exit 1; }
  JDT_GRAPH_UPLOAD=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/r5s40/b$r.log 2>&1 || { tail -5 gpurun_out/r5s40/b$r.log; exit 1; }
  timeout -k 10 120 python bench.py --steps 20 --warmup 25 > gpurun_out/r5s40/c$r.log 2>&1 || { tail -5 gpurun_out/r5s40/c$r.log; exit 1; }
  echo "rep $r: A $(v gpurun_out/r5s40/a$r.log)  B-upload $(v gpurun_out/r5s40/b$r.log)  C-warm25 $(v gpurun_out/r5s40/c$r.log)"
done
echo done
