#!/bin/bash
# One GPU-box session: numerics tests, 1-GPU bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/timeout ends the script.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
stage() { echo "[gpu_check] $(date +%T) $*"; }
fatal_rc() { case "$1" in 0|1) return 1;; *) return 0;; esac; }

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  stage "pytest -m gpu"
  timeout -k 10 ${TEST_TIMEOUT:-600} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; tail -5 "$OUT/pytest_gpu.log"; stage "pytest rc=$rc"
  if fatal_rc $rc; then stage "stopping after fatal rc"; exit $rc; fi
fi
stage "bench"
timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
rc=$?; tail -2 "$OUT/bench.log"; stage "bench rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${SKIP_PROF:-0}" != "1" ]; then
  stage "rocprofv3 kernel stats"
  cd /tmp
  timeout -k 10 ${PROF_TIMEOUT:-300} rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 "$ROOT/bench.py" --steps 200 --warmup 20 ${BENCH_ARGS:-} > "$OUT/prof.log" 2>&1
  rc=$?; tail -3 "$OUT/prof.log"; stage "rocprof rc=$rc"
  find "$OUT/prof" -name "*stats*" | head
fi
