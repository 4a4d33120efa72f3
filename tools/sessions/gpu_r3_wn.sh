#!/bin/bash
# md_bwd: both W_{i+1} parities loaded up front (no load behind the step counter): deep tests,
# benches (compare profiles/r3_dz_split_ab.txt), stamps
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/wn
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_grad_scale_gpu.py tests/test_fused_stage_gpu.py tests/test_deterministic_gpu.py -q -x --timeout 150 --timeout-method thread -k "dz_split or deep or fused_mode or run_ahead or fused_stage or determin or mb_streams" > gpurun_out/wn/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|Error" gpurun_out/wn/pytest.log | tail -8
case $rc in 0) ;; *) exit $rc;; esac
for rep in 1 2; do
  for a in "--num-layers 4" "--num-layers 3" "--strategy pp --hidden-layers 8"; do
    timeout -k 10 150 python bench.py --steps 300 --warmup 30 $a > gpurun_out/wn/b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/wn/b.log; exit 1; }
    echo "rep $rep $a: $(grep '^{' gpurun_out/wn/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
  done
done
timeout -k 10 120 python tools/stamp_deep.py --layers 4 > gpurun_out/wn/stamp.log 2>&1 || { tail -5 gpurun_out/wn/stamp.log; exit 1; }
grep -v amdgpu.ids gpurun_out/wn/stamp.log
