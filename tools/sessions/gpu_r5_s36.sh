# md_bwd AdamW-constant pin: every layer (1) vs only layers whose step counter is the first load (2)
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 JDT_AUTOBUILD=0 && mkdir -p gpurun_out/r5s36 || exit 1
L=jax_distributed_tuts_amd/ops/lib
for rep in 1 2 3; do
  for v in 1 2; do
    cp $L/libjdt_pin$v.so $L/libjdt_kernels.so || exit 1
    timeout -k 10 180 python bench.py --steps 300 --warmup 30 --num-layers 4 > gpurun_out/r5s36/v$v.r$rep.log 2>&1 || exit 1
    echo "rep $rep pin $v 4-layer: $(grep -o '"value": [0-9.]*' gpurun_out/r5s36/v$v.r$rep.log)"
  done
done
