#!/bin/bash
# PMC comparison of the 64x64 (cfg 11) and 128x128 (cfg 14) LDS-DMA GEMM tiles on one shape.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_tiles
mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
for cfg in 11 14; do
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES \
    --kernel-trace --output-format csv -d "$OUT/c$cfg" -o run -- python3 "$ROOT/tools/bench_gemm.py" --cfg $cfg --only "qkv fwd 2k" > "$OUT/c$cfg.log" 2>&1
  rc=$?; echo "[pmc] cfg $cfg rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/c$cfg.log"; exit $rc; }
done
cd $ROOT && timeout -k 10 300 python bench.py --strategy pp --model transformer --merge-microbatches --steps 100 --warmup 10 > gpurun_out/tf.log 2>&1; echo "tf rc=$?"; tail -1 gpurun_out/tf.log | cut -c1-330
