#!/bin/bash
# Round 4 session 10: the tile exchange's start-up self-test at W = 2 / 4 / 8 (shared GPU),
# the DP one-launch tests again, phase stamps of the one-launch N = 2 step, and the
# driver-form bench at N = 2 / 4 (4: three-launch on the shared GPU, grids do not fit).
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s10
timeout -k 10 500 python -u -m pytest tests/test_xgmi_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread \
  -k "tile_exchange or dp_over_xgmi" > gpurun_out/s10/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/s10/pytest.log | tail -12
[ $rc -ne 0 ] && { grep -E "Error|assert|selftest|timed out" gpurun_out/s10/pytest.log | head -30; exit $rc; }
JDT_BACKEND=gloo timeout -k 10 180 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29513 tools/stamp_dp_tx.py > gpurun_out/s10/stamps.log 2>&1 || { tail -20 gpurun_out/s10/stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/s10/stamps.log | tail -16
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print(j["value"], j["ms_per_step"], c.get("step_launches"))'; }
for n in 2 4; do
  for r in 1 2; do
    JDT_BACKEND=gloo timeout -k 10 200 python bench.py --gpus $n --steps 20 --warmup 5 > gpurun_out/s10/b$n.log 2>&1 || { tail -8 gpurun_out/s10/b$n.log; exit 1; }
    echo "N=$n driver form rep $r: $(js gpurun_out/s10/b$n.log)"
  done
done
echo done
