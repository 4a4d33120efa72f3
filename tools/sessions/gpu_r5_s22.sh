# xGMI context churn: self-test failure rate per teardown mode, 4 and 8 ranks sharing the GPU
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 JDT_BACKEND=gloo PYTHONPATH=/root/repo && mkdir -p gpurun_out/r5s22 || exit 1
show() { tail -1 "$1"; grep -h "self-test failed" "$1" | head -8 || true; }
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29731 \
  tools/xgmi_churn.py --iters 12 > gpurun_out/r5s22/w4.log 2>&1 || { echo "w4 exit $?"; tail -20 gpurun_out/r5s22/w4.log; exit 1; }
show gpurun_out/r5s22/w4.log
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29732 \
  tools/xgmi_churn.py --iters 8 > gpurun_out/r5s22/w8.log 2>&1 || { echo "w8 exit $?"; tail -20 gpurun_out/r5s22/w8.log; exit 1; }
show gpurun_out/r5s22/w8.log
