#!/bin/bash
# LN backward: waves-per-workgroup x rows-per-wave sweep, LN tests, transformer step A/B (W=4 R=auto vs new default)
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/ln3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "layernorm" > gpurun_out/ln3/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/ln3/pytest.log; exit 1; }
tail -2 gpurun_out/ln3/pytest.log
timeout -k 10 200 python tools/bench_ln.py > gpurun_out/ln3/bench_ln.log 2>&1 || { echo "bench_ln rc=$?"; tail -5 gpurun_out/ln3/bench_ln.log; exit 1; }
grep ln_bwd gpurun_out/ln3/bench_ln.log
for rep in 1 2; do
for w in 4 0; do
  JDT_LN_WAVES=$w timeout -k 10 200 python bench.py --strategy pp --model transformer --steps 300 --warmup 30 > gpurun_out/ln3/b.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/ln3/b.log; exit 1; }
  echo "waves=$w: $(grep '^{' gpurun_out/ln3/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
done
done
