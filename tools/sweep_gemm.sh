set -u
mkdir -p gpurun_out
for cfg in 1 2 3; do for ex in 2 4 8 16; do
  echo "=== cfg $cfg exact $ex"
  timeout -k 10 120 python tools/bench_gemm.py --cfg $cfg --exact $ex || exit $?
done; done > gpurun_out/sweep.txt 2>&1
echo "=== auto" >> gpurun_out/sweep.txt
timeout -k 10 120 python tools/bench_gemm.py >> gpurun_out/sweep.txt 2>&1
