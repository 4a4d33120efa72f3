#!/bin/bash
# PMC counters of the 4-layer step's kernels (md_fwd / md_bwd variants) from one bench.py run each
# (--num-layers 4 --steps 100).  One counter group per rocprofv3 run, --kernel-trace only.
# Medians per dispatch.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_deep
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 python3 -c "import torch" || exit 1
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
           "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/g$i" -o run -- \
    python3 "$ROOT/bench.py" --steps 100 --warmup 20 --num-layers 4 > "$OUT/g$i.log" 2>&1
  rc=$?; echo "[pmc] group $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/g$i.log"; exit $rc; fi
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
names = {}
for f in glob.glob(f"{out}/g*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if "md_fwd" not in k and "md_bwd" not in k:
            continue
        t = k.split("(")[0].replace("void jdt::", "")
        agg[t][r["Counter_Name"]].append(float(r["Counter_Value"]))
for t, d in sorted(agg.items(), key=lambda kv: -len(next(iter(kv[1].values())))):
    n = len(next(iter(d.values())))
    if n < 20:
        continue   # warmup-only variants
    print(f"== {t}")
    for c, v in sorted(d.items()):
        v = sorted(v)
        print(f"  {c:34s} median {v[len(v)//2]:14.1f}  (n={len(v)})")
PY
