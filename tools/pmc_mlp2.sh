#!/bin/bash
# PMC counters of the fused classifier step kernels (mlp2_fwd / mlp2_bwd), eager
# launches from tools/stamp_mlp2.py (two-launch pair and the run-ahead backward).
# One counter group per rocprofv3 run.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_mlp2
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
# page the torch libraries in first (the first import on a fresh box takes 1-2 minutes,
# which a per-group time limit would otherwise count)
timeout -k 10 300 python3 -c "import torch" || exit 1
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
           "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/g$i" -o run -- \
    python3 "$ROOT/tools/stamp_mlp2.py" --iters 20 > "$OUT/g$i.log" 2>&1
  rc=$?; echo "[pmc] group $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/g$i.log"; exit $rc; fi
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/g*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if "mlp2" not in k:
            continue
        kn = "fwd" if "fwd" in k else ("bwd_run_ahead" if "112, true, true" in k else "bwd")
        agg[kn][r["Counter_Name"]].append(float(r["Counter_Value"]))
for kn, d in agg.items():
    print(f"== mlp2_{kn}")
    for c, v in sorted(d.items()):
        v = sorted(v)
        print(f"  {c:34s} median {v[len(v)//2]:14.1f}  (n={len(v)})")
PY
