#!/bin/bash
# Round 4 session 20: PMC counters of the current headline kernels (tools/pmc_mlp2.sh: one counter
# group per rocprofv3 run, kernel trace only), incl. LDS instructions / bank conflicts.
cd /root/repo && export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash tools/pmc_mlp2.sh > gpurun_out/pmc_r4.txt 2>&1; rc=$?
cat gpurun_out/pmc_r4.txt
exit $rc
