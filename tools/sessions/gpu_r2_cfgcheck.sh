#!/bin/bash
# every BASELINE config's N>1 path on the shared GPU: graph-captured? which transport? steps/s
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 JDT_BACKEND=gloo && mkdir -p gpurun_out/cc
for spec in "2:--num-layers 4" "4:--num-layers 4" "2:--strategy fsdp --num-layers 4" "2:--strategy pp --hidden-layers 8" \
            "4:--strategy pp --hidden-layers 8" "4:--strategy pp --dp 2 --model transformer" "4:--strategy pp --dp 2 --hidden-layers 8" \
            "2:--accum loop" "2:--strategy pp --model transformer"; do
  n=${spec%%:*}; a=${spec#*:}
  timeout -k 10 300 python bench.py --gpus $n --steps 100 --warmup 10 $a > gpurun_out/cc/b.log 2>&1 || { echo "N=$n '$a' rc=$?"; tail -4 gpurun_out/cc/b.log; continue; }
  echo "N=$n '$a': $(grep '^{' gpurun_out/cc/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); d=j["details"]; print(j["value"], j["ms_per_step"], "graph", d["hipgraph"], d["steps_per_graph"], d["comm"], d["xgmi_selftest"])')"
done
