#!/bin/bash
# Entry scripts end to end after the stream schedules (DP loop on 2 streams at 4 layers, one-stage LM on 4 microbatch streams): 1 process, then 4 processes sharing the GPU
# (xGMI kernels between them), incl. the reference-faithful FSDP loop and the GPipe default
# microbatch count; replication checks on the multi-rank runs
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/entry4
export PYTHONUNBUFFERED=1
i=0
run() { i=$((i+1)); timeout -k 10 240 "$@" > gpurun_out/entry4/e$i.log 2>&1 || { echo "FAILED: $*"; tail -30 gpurun_out/entry4/e$i.log; exit 3; }; echo "== $*"; tail -4 gpurun_out/entry4/e$i.log; }
run python data_paral.py
run python data_paral.py --num-layers 4 --check-replication
run python param_sharding.py
run python param_sharding.py --num-layers 4
run python pipeline_parallel.py
run python pipeline_parallel.py --model transformer
export JDT_BACKEND=gloo
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1"
run $TR --master-port 29611 data_paral.py --check-replication
run $TR --master-port 29612 param_sharding.py --check-replication
run $TR --master-port 29613 pipeline_parallel.py --check-replication
run $TR --master-port 29614 pipeline_parallel.py --dp 2 --model transformer --check-replication
run python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29615 pipeline_parallel.py --dp 2 --model transformer --check-replication
