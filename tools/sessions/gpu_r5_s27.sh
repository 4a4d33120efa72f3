# after the persistent headline kernel: whole GPU suite, smoke, the 1-GPU configs that run the
# fused 2-layer engine, the driver form, and the headline's kernel statistics
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s27 || exit 1
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; print(j["value"], j["ms_per_step"], c.get("step_launches", ""))'; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread \
  > gpurun_out/r5s27/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -3 gpurun_out/r5s27/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r5s27/pytest_gpu.log | head -20; fatal $rc && exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5s27/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/r5s27/smoke.log; exit 1; }
echo "smoke ok"
i=0
for a in "" "--optimizer sgd" "--strategy fsdp"; do
  i=$((i+1))
  timeout -k 10 180 python bench.py --steps 300 --warmup 30 $a > gpurun_out/r5s27/b$i.log 2>&1 || { echo "bench '$a' failed"; tail -5 gpurun_out/r5s27/b$i.log; exit 1; }
  echo "== $a: $(js gpurun_out/r5s27/b$i.log)"
done
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/r5s27/d$r.log 2>&1 || { tail -5 gpurun_out/r5s27/d$r.log; exit 1; }
  echo "== driver form $r: $(js gpurun_out/r5s27/d$r.log)"
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r5s27/prof -o headline -- python bench.py --steps 300 --warmup 30 > gpurun_out/r5s27/prof.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/r5s27/prof.log; exit 1; }
find gpurun_out/r5s27/prof -name "*kernel_stats.csv" | head -3
