set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s32
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r6s32
for f in "" "--no-dbias"; do timeout -k 10 120 python tools/stamp_attn.py --batch 16 $f > $O/st.log 2>&1 || { tail -20 $O/st.log; exit 3; }; echo "[$f]"; grep -v amdgpu $O/st.log; done
