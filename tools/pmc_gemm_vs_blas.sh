#!/bin/bash
# PMC: our LDS-DMA GEMM vs hipBLASLt on one shape (tools/bench_gemm.py --only SHAPE runs both)
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$ROOT/gpurun_out/pmcb; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
SHAPE=${SHAPE:-fc2 dX 2k}
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 $ROOT/tools/bench_gemm.py --only "$SHAPE" > $OUT/p$i.log 2>&1
  rc=$?; echo "[pmc] pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/p$i.log; exit $rc; }
done
