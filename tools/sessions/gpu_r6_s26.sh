set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s26
export PYTHONUNBUFFERED=1 TMPDIR=/tmp JDT_BACKEND=gloo
O=gpurun_out/r6s26
for n in 2 4; do for st in dp fsdp; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --strategy $st --steps 20 --warmup 5 > $O/b_${st}_$n.log 2>&1 || { echo "N=$n $st failed"; tail -30 $O/b_${st}_$n.log; exit 3; }
  echo "N=$n $st: $(grep '"metric"' $O/b_${st}_$n.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'], d['config'].get('parallelism'), str(d.get('details',{}).get('autotune',{}).get('chosen','')))")"
done; done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29510 bench.py --gpus 2 --strategy pp --hidden-layers 8 --steps 20 --warmup 5 > $O/b_pp_2.log 2>&1 || { echo "N=2 pp failed"; tail -30 $O/b_pp_2.log; exit 3; }
echo "N=2 pp: $(grep '"metric"' $O/b_pp_2.log | tail -1 | cut -c1-200)"
