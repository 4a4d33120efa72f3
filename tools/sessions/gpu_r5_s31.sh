# persistent multi-step replay: direct kernel launch vs the one-node graph, driver form, alternating
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s31 || exit 1
for rep in 1 2 3 4; do
  for d in 1 0; do
    JDT_PST_DIRECT=$d timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/r5s31/d$d.r$rep.log 2>&1 || { echo "bench exit"; exit 1; }
    echo "rep $rep direct $d: $(grep -o '"value": [0-9.]*' gpurun_out/r5s31/d$d.r$rep.log)"
  done
done
for d in 1 0; do
  JDT_PST_DIRECT=$d timeout -k 10 120 python bench.py --steps 300 --warmup 30 > gpurun_out/r5s31/l$d.log 2>&1 || exit 1
  echo "direct $d 300 steps: $(grep -o '"value": [0-9.]*' gpurun_out/r5s31/l$d.log)"
done
