cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s32 || exit 1
for rep in 1 2 3; do
  timeout -k 10 180 python bench.py --steps 300 --warmup 30 --num-layers 4 > gpurun_out/r5s32/l4.r$rep.log 2>&1 || exit 1
  echo "rep $rep 4-layer: $(grep -o '"value": [0-9.]*' gpurun_out/r5s32/l4.r$rep.log)"
done
timeout -k 10 180 python bench.py --steps 300 --warmup 30 --strategy pp --hidden-layers 8 > gpurun_out/r5s32/pp8.log 2>&1 || exit 1
echo "GPipe-8 one stage: $(grep -o '"value": [0-9.]*' gpurun_out/r5s32/pp8.log)"
