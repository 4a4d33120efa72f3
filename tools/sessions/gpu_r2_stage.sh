#!/bin/bash
# fused GPipe stage: tests, full GPU suite, PP benches (+ rocprofv3 kernel stats of the PP step)
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_fused_stage_gpu.py tests/test_reference_loss_fn.py -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_stage.log 2>&1
rc=$?; echo "stage rc=$rc"; grep -E "PASS|FAIL|Error" gpurun_out/pytest_stage.log | tail -24
fatal $rc && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "all-gpu rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
fatal $rc && exit $rc
for a in "--strategy pp --hidden-layers 8" "--strategy pp --hidden-layers 8 --merge-microbatches" "--num-layers 4" "--strategy fsdp --num-layers 4"; do
  timeout -k 10 200 python bench.py $a --steps 500 > gpurun_out/b.log 2>&1; rc=$?
  echo "bench [$a] rc=$rc"; tail -1 gpurun_out/b.log | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value'], j['ms_per_step'], j['config'].get('parallelism'))"
  fatal $rc && exit $rc
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pp -o pp -- python bench.py --strategy pp --hidden-layers 8 --steps 200 > gpurun_out/prof_pp.log 2>&1
echo "prof rc=$?"; find gpurun_out/prof_pp -name "*kernel_stats.csv" | head -3
