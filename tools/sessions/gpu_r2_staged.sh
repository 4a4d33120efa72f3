#!/bin/bash
# staged DP all-reduce: xGMI tests + full GPU suite, shared-GPU 2/4-rank benches, transformer profile
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_xgmi_gpu.py tests/test_grad_scale_gpu.py tests/test_deterministic_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_xg.log 2>&1
rc=$?; echo "xgmi rc=$rc"; tail -3 gpurun_out/pytest_xg.log; fatal $rc && exit $rc; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "all-gpu rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; fatal $rc && exit $rc
for n in 2 4; do
  JDT_BACKEND=gloo timeout -k 10 200 python bench.py --gpus $n --steps 200 --warmup 20 > gpurun_out/bench${n}_gloo.log 2>&1; rc=$?
  echo "bench$n rc=$rc"; grep '^{' gpurun_out/bench${n}_gloo.log | python -c "import json,sys; j=json.loads(sys.stdin.read()); d=j['details']; print(j['value'], j['ms_per_step'], d['comm'], d['xgmi_selftest'], d['collective_ms_p50'], d['comm_sweep'])"
  fatal $rc && exit $rc
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tf -o tf -- python bench.py --strategy pp --model transformer --merge-microbatches --steps 60 --warmup 5 > gpurun_out/prof_tf.log 2>&1
echo "prof rc=$?"; tail -1 gpurun_out/prof_tf.log | cut -c1-200
