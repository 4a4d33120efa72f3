set -u
mkdir -p gpurun_out
for cfg in 10 11 12 13; do for sp in 1 2 4; do
  echo "=== cfg $cfg splits $sp"
  timeout -k 10 120 python tools/bench_gemm.py --cfg $cfg --splits $sp || exit $?
done; done > gpurun_out/sweep.txt 2>&1
echo "=== auto" >> gpurun_out/sweep.txt
timeout -k 10 120 python tools/bench_gemm.py >> gpurun_out/sweep.txt 2>&1
