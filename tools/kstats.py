"""Summarise a rocprofv3 kernel_stats.csv: per-kernel calls, mean us, share, and per-step
totals.  Usage: python tools/kstats.py CSV [steps] [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{sys.argv[1]}: {len(rows)} kernels, total {tot / 1e6:.2f} ms" + (f", {tot / 1e3 / steps:.1f} us/step over {steps} steps" if steps else ""))
for r in rows[:top]:
    calls, avg = int(r["Calls"]), float(r["AverageNs"]) / 1e3
    ps = f" {calls / steps:6.1f}/step {calls * avg / steps:8.1f} us/step" if steps else ""
    print(f'{r["Name"][:80]:80s} {calls:>6} {avg:8.2f}us {float(r["Percentage"]):6.2f}%{ps}')
