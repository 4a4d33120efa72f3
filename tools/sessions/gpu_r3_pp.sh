# GPipe microbatch-count table: per-stage tick costs on one GPU
# (tools/pp_schedule.py), then the shared-GPU rehearsal of PP2 / PP4 (N processes
# time-share cuda:0, xGMI inbox hand-off between them) at several microbatch counts.
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python tools/pp_schedule.py --reps 200 --out gpurun_out/pp_schedule.json > gpurun_out/pp_schedule.log 2>&1 \
  || { echo "pp_schedule failed"; tail -30 gpurun_out/pp_schedule.log; exit 3; }
cat gpurun_out/pp_schedule.log
export JDT_BACKEND=gloo
: > gpurun_out/pp_shared.jsonl
for n in 2 4; do
  for mbc in 1 2 4 8 16; do
    timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29600 + n * 20 + mbc)) bench.py --gpus $n --steps 100 --warmup 20 --strategy pp \
      --hidden-layers 8 --microbatches $mbc > gpurun_out/pp_m.log 2>&1 || { echo "mlp N=$n mb=$mbc failed"; tail -30 gpurun_out/pp_m.log; exit 3; }
    echo "== mlp pp$n n_mb=$mbc"; grep '"metric"' gpurun_out/pp_m.log | tee -a gpurun_out/pp_shared.jsonl | cut -c1-160
  done
  for mbc in 1 2 4 8; do
    timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29700 + n * 20 + mbc)) bench.py --gpus $n --steps 50 --warmup 10 --strategy pp \
      --model transformer --lm-batch 8 --microbatches $mbc > gpurun_out/pp_t.log 2>&1 || { echo "lm N=$n mb=$mbc failed"; tail -30 gpurun_out/pp_t.log; exit 3; }
    echo "== lm pp$n n_mb=$mbc"; grep '"metric"' gpurun_out/pp_t.log | tee -a gpurun_out/pp_shared.jsonl | cut -c1-160
  done
done
