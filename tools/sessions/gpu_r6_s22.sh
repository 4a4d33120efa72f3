set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s22
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s22
for gm in -1 0 2 4 8; do
  timeout -k 10 200 python tools/bench_lm_gemms.py --gm $gm > $O/g$gm.log 2>&1 || { tail -20 $O/g$gm.log; exit 3; }
  echo "== gm $gm"; cat $O/g$gm.log | grep -v amdgpu.ids
done
