set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in 0 1 0 1; do
  echo "== JDT_GROUP_SPLIT=$v"; JDT_GROUP_SPLIT=$v timeout -k 10 150 python bench.py --strategy pp --model transformer --steps 300 --warmup 30 | tail -1 | cut -c80-180
done
cd /tmp
for v in 0 1; do
  JDT_GROUP_SPLIT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/gs$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --strategy pp --model transformer --steps 100 --warmup 10 > $GRAFT_REPO_ROOT/gpurun_out/gs$v.log 2>&1 || exit 3
done
