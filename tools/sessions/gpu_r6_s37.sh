set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s37
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s37
timeout -k 10 200 python tools/bench_lm_gemms.py > $O/g.log 2>&1 || { tail -20 $O/g.log; exit 3; }; grep -v amdgpu $O/g.log
