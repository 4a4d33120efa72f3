#!/bin/bash
# Entry scripts end to end after the run-ahead changes: 1 process (run-ahead graphs), then
# 4 processes sharing the GPU (two-launch + xGMI)
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/entry
export PYTHONUNBUFFERED=1
i=0
run() { i=$((i+1)); timeout -k 10 240 "$@" > gpurun_out/entry/e$i.log 2>&1 || { echo "FAILED: $*"; tail -30 gpurun_out/entry/e$i.log; exit 3; }; echo "== $*"; tail -4 gpurun_out/entry/e$i.log; }
run python data_paral.py
run python data_paral.py --num-layers 4 --check-replication
run python data_paral.py --deterministic
run python param_sharding.py --num-layers 4
run python pipeline_parallel.py
export JDT_BACKEND=gloo
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29611"
run $TR data_paral.py --check-replication
run $TR param_sharding.py
