# Rehearse bench.py's N>1 path on the 1-GPU box: N processes share cuda:0, gloo
# bootstrap, xGMI P2P kernels between the processes.  Timings are NOT multi-GPU
# numbers (the ranks time-share one GPU); this checks the code path end to end.
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export JDT_BACKEND=gloo PYTHONUNBUFFERED=1
for n in ${MP_NS:-2 4}; do
  for a in "" "--strategy fsdp" "--strategy pp --hidden-layers 8"; do
    timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29500 + n)) bench.py --gpus $n --steps 100 --warmup 10 $a > gpurun_out/mp_$n.log 2>&1 || { echo "N=$n $a failed"; tail -30 gpurun_out/mp_$n.log; exit 3; }
    echo "== N=$n $a"; grep '"metric"' gpurun_out/mp_$n.log | cut -c1-120; grep -o '"comm": "[a-z]*"' gpurun_out/mp_$n.log
  done
done
