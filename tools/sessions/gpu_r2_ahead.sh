#!/bin/bash
# Run-ahead backward (one launch per step): GPU equivalence tests, then in-model A/B
# (JDT_MLP2_AHEAD=0/1, alternating) at the driver's short region and at 300 steps.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/ahead
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "run_ahead or loop_kernel or fused_mlp_step or deterministic" > gpurun_out/ahead/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|PASS|FAIL|Error" gpurun_out/ahead/pytest.log | tail -15
[ $rc -ne 0 ] && exit $rc
out=gpurun_out/ahead/ab.txt; : > $out
val() { grep '^{' "$1" | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["details"]["final_loss"])'; }
for rep in 1 2; do
  for ah in 0 1; do
    for st in "20 5" "300 30"; do
      set -- $st
      JDT_MLP2_AHEAD=$ah timeout -k 10 120 python bench.py --steps $1 --warmup $2 > gpurun_out/ahead/b.log 2>&1; rc=$?
      [ $rc -ne 0 ] && { echo "ahead=$ah rc=$rc"; tail -5 gpurun_out/ahead/b.log; exit $rc; }
      echo "rep $rep ahead=$ah steps=$1: $(val gpurun_out/ahead/b.log)" | tee -a $out
    done
  done
done
timeout -k 10 120 python tools/stamp_mlp2.py > gpurun_out/ahead/stamps.txt 2>&1 && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ahead/prof -o run -- python3 bench.py --steps 300 --warmup 30 > gpurun_out/ahead/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; find gpurun_out/ahead/prof -name "*kernel_stats.csv" | head -2
