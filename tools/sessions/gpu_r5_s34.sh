cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s34 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_grad_scale_gpu.py tests/test_pp_chain_gpu.py \
  -k "deep or md or adam or pipeline or chain or fsdp" > gpurun_out/r5s34/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r5s34/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r5s34/tests.log | head; exit 1; }
for rep in 1 2 3; do
  timeout -k 10 180 python bench.py --steps 300 --warmup 30 --num-layers 4 > gpurun_out/r5s34/l4.r$rep.log 2>&1 || exit 1
  echo "rep $rep 4-layer: $(grep -o '"value": [0-9.]*' gpurun_out/r5s34/l4.r$rep.log)"
done
timeout -k 10 180 python bench.py --steps 300 --warmup 30 --strategy pp --hidden-layers 8 > gpurun_out/r5s34/pp8.log 2>&1 || exit 1
echo "GPipe-8 one stage: $(grep -o '"value": [0-9.]*' gpurun_out/r5s34/pp8.log)"
