set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r6s40
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r6s40
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "wpass|adamw_ranges" --output-format csv -d $O/fetch -o f -- python3 $GRAFT_REPO_ROOT/bench.py --strategy pp --model transformer --steps 20 --warmup 5 > $O/fetch.log 2>&1 || { tail -20 $O/fetch.log; exit 3; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "wpass|adamw_ranges" --output-format csv -d $O/write -o w -- python3 $GRAFT_REPO_ROOT/bench.py --strategy pp --model transformer --steps 20 --warmup 5 > $O/write.log 2>&1 || { tail -20 $O/write.log; exit 3; }
cd $GRAFT_REPO_ROOT
python - <<'PY'
import csv, glob, collections
for tag in ("fetch", "write"):
    fs = glob.glob(f"gpurun_out/r6s40/{tag}/*counter_collection.csv")
    if not fs: print(tag, "no csv", glob.glob(f"gpurun_out/r6s40/{tag}/*")); continue
    r = list(csv.DictReader(open(fs[0])))
    print(tag, "cols", list(r[0].keys())[:30])
    agg = collections.defaultdict(list)
    for x in r:
        agg[(x.get("Kernel_Name", "")[:40], x.get("Counter_Name"))].append(float(x.get("Counter_Value", 0)))
    for k, v in agg.items():
        print(tag, k, len(v), "median", sorted(v)[len(v)//2])
PY
