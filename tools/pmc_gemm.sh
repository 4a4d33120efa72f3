#!/bin/bash
# PMC counters of the LDS-DMA GEMM on two transformer shapes: a K-contiguous x
# transposed-B forward (qkv) and a both-transposed weight gradient (fc1 dW).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_gemm
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAVE_CYCLES SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/g$i" -o run -- \
    python3 "$ROOT/tools/bench_gemm.py" --only "qkv fwd,fc1 dW,fc2 dX" > "$OUT/g$i.log" 2>&1
  rc=$?; echo "[pmc] group $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/g$i.log"; exit $rc; fi
done
