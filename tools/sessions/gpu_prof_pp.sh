set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_pp -o run -- python3 $R/bench.py --steps 60 --warmup 10 --strategy pp --hidden-layers 8 > $R/gpurun_out/prof_pp.log 2>&1 || { tail -20 $R/gpurun_out/prof_pp.log; exit 3; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_lm -o run -- python3 $R/bench.py --steps 20 --warmup 5 --strategy pp --model transformer > $R/gpurun_out/prof_lm.log 2>&1 || { tail -20 $R/gpurun_out/prof_lm.log; exit 3; }
find $R/gpurun_out/prof_pp $R/gpurun_out/prof_lm -name "*kernel_stats*"
