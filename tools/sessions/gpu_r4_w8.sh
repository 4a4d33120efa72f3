#!/bin/bash
# Round 4: 8 ranks sharing the one GPU (gloo bootstrap, xGMI IPC kernels between the
# processes): the W = 8 kernel instantiations (xg_kernel<8>, xg_oneshot_kernel<8>,
# xg_seg_kernel<8>, xg_fsdp_kernel<8>, the 8-stage inbox schedule) and every BASELINE
# config's layout at 8 ranks.  Code-path checks, not link numbers.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/w8
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_rccl_capture_gpu.py tests/test_reference_loss_fn.py -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/w8/pytest_rccl.log 2>&1
rc=$?; echo "pytest rccl-capture + scan-cache rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/w8/pytest_rccl.log | tail -20
[ $rc -ne 0 ] && { tail -30 gpurun_out/w8/pytest_rccl.log; exit $rc; }
timeout -k 10 900 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/w8/pytest_xgmi.log 2>&1
rc=$?; echo "pytest xgmi rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/w8/pytest_xgmi.log | tail -40
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_grad_scale_gpu.py -x -v -k xgmi --timeout 240 --timeout-method thread \
  > gpurun_out/w8/pytest_scale.log 2>&1
rc=$?; echo "pytest grad-scale rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/w8/pytest_scale.log | tail -20
[ $rc -ne 0 ] && exit $rc
export JDT_BACKEND=gloo
: > gpurun_out/w8/bench8.jsonl
i=0
for a in "" "--num-layers 4" "--strategy fsdp" "--strategy fsdp --num-layers 4" "--strategy pp --hidden-layers 8" \
         "--strategy pp --dp 2 --model transformer"; do
  i=$((i+1))
  timeout -k 10 240 python bench.py --gpus 8 --steps 100 --warmup 10 $a > gpurun_out/w8/b$i.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "N=8 '$a' rc=$rc"; tail -8 gpurun_out/w8/b$i.log; fatal $rc && exit $rc; continue; }
  echo "== N=8 $a: $(grep '^{' gpurun_out/w8/b$i.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["details"]["comm"], j["details"]["xgmi_selftest"], j["details"]["hipgraph"])')"
  grep '^{' gpurun_out/w8/b$i.log >> gpurun_out/w8/bench8.jsonl
done
for s in "data_paral.py --num-layers 4" "param_sharding.py --num-layers 4" "pipeline_parallel.py" \
         "pipeline_parallel.py --dp 2 --model transformer"; do
  i=$((i+1))
  timeout -k 10 240 python $s --gpus 8 --check-replication > gpurun_out/w8/e$i.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "entry '$s' rc=$rc"; tail -8 gpurun_out/w8/e$i.log; fatal $rc && exit $rc; continue; }
  echo "== entry $s --gpus 8 --check-replication:"; grep -iE "replicat|loss|accuracy" gpurun_out/w8/e$i.log | tail -4
done
echo done
