#!/bin/bash
# PMC counters of the persistent headline kernel (mlp2_pst_kernel) against the one-step
# run-ahead kernel, both from one bench.py run (--steps 200: one 200-step persistent launch;
# the warmup's 1-step graphs replay the one-step kernel).  One counter group per rocprofv3 run,
# --kernel-trace only.  Persistent-kernel counters are reported per step (/ 200).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_pst
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
    python3 "$ROOT/bench.py" --steps 200 --warmup 30 > "$OUT/g$i.log" 2>&1
  rc=$?; echo "[pmc] group $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/g$i.log"; exit $rc; fi
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
one = collections.defaultdict(list)
pst = collections.defaultdict(list)
for f in glob.glob(f"{out}/g*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        v = float(r["Counter_Value"])
        if "mlp2_pst_kernel" in k:
            pst[r["Counter_Name"]].append(v)
        elif "mlp2_bwd_kernel" in k and "112, true, true" in k:
            one[r["Counter_Name"]].append(v)
print(f"{'counter':34s} {'one-step run-ahead (median/launch)':>36s} {'persistent (per step, /200)':>30s}")
for c in sorted(set(one) | set(pst)):
    a = sorted(one.get(c, [0.0]))
    b = max(pst.get(c, [0.0]))   # the 200-step dispatch (the other is the n = 0 warm no-op)
    print(f"{c:34s} {a[len(a)//2]:36.1f} {b / 200:30.1f}")
PY
