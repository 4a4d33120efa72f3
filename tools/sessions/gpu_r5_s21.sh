#!/bin/bash
# Round 5 session 21: after the collective teardown -- the autotune's repeated trainer
# builds at 4 and 8 shared ranks (DP / FSDP), checking every log for xGMI self-test failures.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1 JDT_BACKEND=gloo && mkdir -p gpurun_out/r5s21
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
js() { grep '^{' $1 | python -c 'import json,sys; j=json.loads(sys.stdin.read()); c=j["config"]; a=j["details"].get("autotune") or {}; print(j["value"], j["ms_per_step"], c.get("step_launches", ""), [(x["name"], x.get("us_per_step")) for s in a.get("stages", []) for x in s["candidates"]])'; }
i=0
for r in 1 2; do for n in 4 8; do for st in "--strategy fsdp" ""; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --gpus $n --steps 200 --warmup 20 $st > gpurun_out/r5s21/r$i.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "N=$n $st rc=$rc"; tail -5 gpurun_out/r5s21/r$i.log; fatal $rc && exit $rc; continue; }
  echo "== run $r N=$n $st: $(js gpurun_out/r5s21/r$i.log) selftest-failures=$(grep -c 'self-test failed' gpurun_out/r5s21/r$i.log)"
done; done; done
