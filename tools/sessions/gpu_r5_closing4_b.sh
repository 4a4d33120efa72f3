#!/bin/bash
# Round 5 closing run 4, part b (final tree; part a: gpu_r5_closing4.sh): DP and FSDP at N = 2 / 4 / 8 ranks sharing
# the GPU (with their autotune tables); GPipe 2 / 4 stages; the entry scripts at 2 and 8 ranks
# with --check-replication.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5close4b
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print(j["value"], j["ms_per_step"], c.get("step_launches", ""))'; }
export JDT_BACKEND=gloo
i=0
for n in 2 4 8; do for st in "" "--strategy fsdp" "--num-layers 4" "--strategy fsdp --num-layers 4"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --gpus $n --steps 200 --warmup 20 $st > gpurun_out/r5close4b/n${n}_$i.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "N=$n $st rc=$rc"; tail -5 gpurun_out/r5close4b/n${n}_$i.log; fatal $rc && exit $rc; continue; }
  echo "== N=$n shared $st: $(js gpurun_out/r5close4b/n${n}_$i.log)"
  grep '^{' gpurun_out/r5close4b/n${n}_$i.log >> gpurun_out/r5close4b/all_b.jsonl
done; done
for n in 2 4; do
  timeout -k 10 300 python bench.py --gpus $n --strategy pp --hidden-layers $n --steps 200 --warmup 20 > gpurun_out/r5close4b/pp$n.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "PP$n rc=$rc"; tail -5 gpurun_out/r5close4b/pp$n.log; fatal $rc && exit $rc; continue; }
  echo "== GPipe $n stages shared: $(js gpurun_out/r5close4b/pp$n.log)"
  grep '^{' gpurun_out/r5close4b/pp$n.log >> gpurun_out/r5close4b/all_b.jsonl
done
for s in "data_paral.py --gpus 2" "param_sharding.py --gpus 2" "data_paral.py --gpus 8 --num-layers 4" "param_sharding.py --gpus 8 --num-layers 4" \
         "pipeline_parallel.py --gpus 8" "pipeline_parallel.py --gpus 8 --dp 2 --model transformer"; do
  i=$((i+1))
  timeout -k 10 300 python $s --check-replication > gpurun_out/r5close4b/e$i.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "entry '$s' rc=$rc"; tail -8 gpurun_out/r5close4b/e$i.log; fatal $rc && exit $rc; continue; }
  echo "== entry $s --check-replication:"; grep -iE "replicat|loss|accuracy" gpurun_out/r5close4b/e$i.log | tail -3
done
echo done
