set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s31
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s31
for b in 16 2; do timeout -k 10 120 python tools/stamp_attn.py --batch $b > $O/st$b.log 2>&1 || { tail -20 $O/st$b.log; exit 3; }; grep -v amdgpu $O/st$b.log; done
timeout -k 10 300 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py -k "attn" > $O/t.log 2>&1; tail -1 $O/t.log
