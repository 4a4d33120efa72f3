# driver-form headline (--steps 20 --warmup 5): steps per captured graph vs the fixed cost of the timed region
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s24 || exit 1
for rep in 1 2 3; do
  for spg in 20 10 5 2 1; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --steps-per-graph $spg > gpurun_out/r5s24/s$spg.r$rep.log 2>&1 \
      || { echo "spg $spg exit $?"; tail -5 gpurun_out/r5s24/s$spg.r$rep.log; exit 1; }
    echo "rep $rep spg $spg: $(grep -o '"value": [0-9.]*' gpurun_out/r5s24/s$spg.r$rep.log)"
  done
done
