#!/bin/bash
# Full GPU suite (run-ahead AdamW scale probe, FSDP loop fix, 32x32 MFMA tiles), LM benches with the
# round-3 GEMM table, shared-GPU PP rehearsals at the new default microbatch count, per-mb LM profile
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 && mkdir -p gpurun_out/s3
JDT_ORACLE_LOG=gpurun_out/s3/oracle.jsonl timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/s3/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|Error" gpurun_out/s3/pytest.log | tail -8
case $rc in 0) ;; *) exit $rc;; esac
: > gpurun_out/s3/all.jsonl
for a in "--strategy pp --model transformer" "--strategy pp --model transformer --microbatch-passes" "" "--strategy fsdp --accum loop"; do
  timeout -k 10 180 python bench.py --steps 200 --warmup 20 $a > gpurun_out/s3/b.log 2>&1 || { echo "bench '$a' failed"; tail -5 gpurun_out/s3/b.log; exit 1; }
  echo "== $a: $(grep '^{' gpurun_out/s3/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
  grep '^{' gpurun_out/s3/b.log >> gpurun_out/s3/all.jsonl
done
export JDT_BACKEND=gloo
for n in 2 4; do
  for a in "--strategy pp --hidden-layers 8" "--strategy pp --hidden-layers 8 --microbatches 4"; do
    timeout -k 10 240 python bench.py --gpus $n --steps 100 --warmup 10 $a > gpurun_out/s3/b.log 2>&1 || { echo "N=$n '$a' failed"; tail -5 gpurun_out/s3/b.log; exit 1; }
    echo "== N=$n $a: $(grep '^{' gpurun_out/s3/b.log | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"], j["config"]["num_microbatches"])')"
    grep '^{' gpurun_out/s3/b.log >> gpurun_out/s3/all.jsonl
  done
done
unset JDT_BACKEND
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s3/prof_lmmb -o run -- \
  python3 bench.py --strategy pp --model transformer --microbatch-passes --steps 100 --warmup 10 > gpurun_out/s3/prof.log 2>&1 || exit 1
