# N=4 FSDP bench (4 ranks sharing the GPU) x 8: xGMI self-test failure diagnostics
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 JDT_BACKEND=gloo && mkdir -p gpurun_out/r5s23 || exit 1
for i in 1 2 3 4 5 6 7 8 9 10 11 12; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port $((29740 + i)) bench.py --gpus 4 --steps 200 --warmup 20 --strategy fsdp > gpurun_out/r5s23/r$i.log 2>&1 \
    || { echo "run $i exit $?"; tail -5 gpurun_out/r5s23/r$i.log; exit 1; }
  echo "== run $i: $(grep -c 'self-test failed' gpurun_out/r5s23/r$i.log) failures"
  grep -h "self-test failed" gpurun_out/r5s23/r$i.log || true
done
timeout -k 10 120 python -u -m pytest -x -v --timeout 100 --timeout-method thread tests/test_ipc_pool_gpu.py 2>&1 | tail -3
