# persistent run-ahead headline kernel: correctness, then driver-form / 300-step A/B
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/r5s25 || exit 1
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_mlp2_persistent_gpu.py \
  > gpurun_out/r5s25/pst_tests.log 2>&1; rc=$?; tail -8 gpurun_out/r5s25/pst_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "ahead or fused_mlp" \
  > gpurun_out/r5s25/ahead_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r5s25/ahead_tests.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for pst in 1 0; do
    JDT_MLP2_PST=$pst timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/r5s25/d$pst.r$rep.log 2>&1 || { echo "bench exit"; exit 1; }
    echo "rep $rep pst $pst driver form: $(grep -o '"value": [0-9.]*' gpurun_out/r5s25/d$pst.r$rep.log)"
  done
done
for pst in 1 0; do
  JDT_MLP2_PST=$pst timeout -k 10 120 python bench.py --steps 300 --warmup 50 > gpurun_out/r5s25/l$pst.log 2>&1 || { echo "bench exit"; exit 1; }
  echo "pst $pst 300 steps: $(grep -o '"value": [0-9.]*' gpurun_out/r5s25/l$pst.log)"
done
