#!/bin/bash
# PMC counter profile of the headline step (separate rocprofv3 runs per counter
# group; counters only with --kernel-trace/--stats, never with trace domains).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAVE_CYCLES"; do
  # (TCC_*/FETCH_SIZE derived counters aborted the profiler on this image -- left out)
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/g$i" -o run -- \
    python3 "$ROOT/bench.py" --steps 40 --warmup 5 ${BENCH_ARGS:-} > "$OUT/g$i.log" 2>&1
  rc=$?; echo "[pmc] group $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/g$i.log"; exit $rc; fi
done
