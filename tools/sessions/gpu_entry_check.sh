# Entry scripts end to end on the GPU box: 1 process, then 4 processes sharing
# the GPU (gloo bootstrap, xGMI kernels between them).
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() { timeout -k 10 240 "$@" > gpurun_out/entry.log 2>&1 || { echo "FAILED: $*"; tail -30 gpurun_out/entry.log; exit 3; }; tail -4 gpurun_out/entry.log; }
run python data_paral.py --accum kernel
run python param_sharding.py
run python pipeline_parallel.py
run python pipeline_parallel.py --model transformer --steps 3
export JDT_BACKEND=gloo
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29611"
run $TR data_paral.py --accum kernel
run $TR param_sharding.py
run $TR pipeline_parallel.py --dp 2
run $TR pipeline_parallel.py --dp 2 --model transformer --steps 3
