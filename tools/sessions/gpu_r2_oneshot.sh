#!/bin/bash
# One-shot xGMI all-reduce: the xGMI collective tests (2 and 4 ranks sharing the GPU), then the
# comm sweep with 2 ranks (one-shot vs two-shot at <= 256 KiB)
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/oneshot
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_xgmi_gpu.py > gpurun_out/oneshot/pytest.log 2>&1
rc=$?; echo "xgmi tests rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/oneshot/pytest.log | tail -14; [ $rc -ne 0 ] && exit $rc
for n in 2 4; do
  JDT_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) \
    tools/bench_comm.py --max-bytes 4194304 --iters 20 > gpurun_out/oneshot/comm$n.log 2>&1
  rc=$?; echo "comm N=$n rc=$rc"; grep '^{' gpurun_out/oneshot/comm$n.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
done
exit 0
