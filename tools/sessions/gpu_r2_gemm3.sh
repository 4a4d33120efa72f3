#!/bin/bash
# 128x128 tile diagnosis: timings of cfg 11/12/14 on the 2k shapes + PMC of cfg 14 on one shape
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd $ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/g3
S="fc1 fwd 2k,fc2 dX 2k,qkv fwd 2k,fc2 fwd 2k,fc1 dW 2k,out fwd"
for c in 11 12 14; do
  timeout -k 10 120 python tools/bench_gemm.py --cfg $c --only "$S" --json gpurun_out/g3/cfg$c.json > gpurun_out/g3/cfg$c.log 2>&1 || { echo "cfg $c rc=$?"; tail -3 gpurun_out/g3/cfg$c.log; exit 1; }
done
echo timings done
cd /tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CU_CYCLES \
  --kernel-trace --output-format csv -d $ROOT/gpurun_out/g3/pmc14 -o run -- python3 $ROOT/tools/bench_gemm.py --cfg 14 --only "fc1 fwd 2k" > $ROOT/gpurun_out/g3/pmc14.log 2>&1
echo "pmc rc=$?"
