#!/bin/bash
# SGD through the entry script (1 GPU: fused) and the 2-rank shared-GPU bench (mode 0 + xGMI)
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/sgde; export PYTHONUNBUFFERED=1
timeout -k 10 240 python data_paral.py --optimizer sgd > gpurun_out/sgde/e1.log 2>&1 || { tail -20 gpurun_out/sgde/e1.log; exit 3; }
tail -3 gpurun_out/sgde/e1.log
JDT_BACKEND=gloo timeout -k 10 240 python bench.py --gpus 2 --optimizer sgd --steps 100 --warmup 10 > gpurun_out/sgde/b2.log 2>&1 || { tail -20 gpurun_out/sgde/b2.log; exit 3; }
grep '^{' gpurun_out/sgde/b2.log | cut -c1-200
