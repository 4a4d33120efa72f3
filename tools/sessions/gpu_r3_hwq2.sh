#!/bin/bash
# GPU_MAX_HW_QUEUES=2 with the stream count capped at the queue count (LM on 2 streams), once
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/hwq2
GPU_MAX_HW_QUEUES=2 timeout -k 10 180 python bench.py --steps 200 --warmup 20 --strategy pp --model transformer > gpurun_out/hwq2/b.log 2>&1 || { echo "bench failed rc=$?"; tail -5 gpurun_out/hwq2/b.log; exit 1; }
echo "hwq 2 LM: $(grep '^{' gpurun_out/hwq2/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["config"]["single_stage_mode"])')"
timeout -k 10 180 python bench.py --steps 200 --warmup 20 --strategy pp --model transformer > gpurun_out/hwq2/b4.log 2>&1 || { echo "bench (default queues) failed"; tail -5 gpurun_out/hwq2/b4.log; exit 1; }
echo "default queues LM: $(grep '^{' gpurun_out/hwq2/b4.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["config"]["single_stage_mode"])')"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/hwq2/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/hwq2/smoke.log; exit 1; }
tail -1 gpurun_out/hwq2/smoke.log
