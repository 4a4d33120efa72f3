"""Concurrency profile of a rocprofv3 kernel trace (``--kernel-trace`` CSV): over the
window of the last ``n`` complete steps (a step = the span between consecutive launches of
the ``marker`` kernel), the wall time with 0, 1, 2, ... kernels running, the summed kernel
time and launches per step, and the top kernels by summed time.

    python tools/ktimeline.py TRACE.csv|RESULTS.db [--marker NAME] [--steps N]

Without --marker the window is the whole trace after the first 20 % (warm-up)."""
from __future__ import annotations

import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default=None, help="substring of the kernel that starts each step")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    if a.trace.endswith(".db"):   # rocprofv3's default rocpd (sqlite) output
        import sqlite3

        con = sqlite3.connect(a.trace)
        ks = sorted((int(s), int(e), n) for s, e, n in con.execute("select start, end, name from kernels"))
    else:
        rows = list(csv.DictReader(open(a.trace)))
        ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    if a.marker:
        marks = [s for s, _, n in ks if a.marker in n]
        marks = marks[-(a.steps + 1):]
        t0, t1 = marks[0], marks[-1]
        nsteps = len(marks) - 1
    else:
        t0 = ks[len(ks) // 5][0]
        t1 = ks[-1][1]
        nsteps = 1
    win = [(max(s, t0), min(e, t1), n) for s, e, n in ks if e > t0 and s < t1]
    ev = []
    for s, e, _ in win:
        ev.append((s, 1))
        ev.append((e, -1))
    ev.sort()
    hist = collections.Counter()
    cur, last = 0, t0
    for t, d in ev:
        hist[cur] += t - last
        cur += d
        last = t
    hist[cur] += t1 - last
    span = t1 - t0
    tot = sum(e - s for s, e, _ in win)
    print(f"window {span / 1e3 / nsteps:.1f} us/step over {nsteps} steps; {len(win) / nsteps:.1f} launches/step; "
          f"summed kernel time {tot / 1e3 / nsteps:.1f} us/step (x{tot / span:.2f} overlap)")
    for k in sorted(hist):
        print(f"  {k} running: {hist[k] / 1e3 / nsteps:8.1f} us/step ({100 * hist[k] / span:5.1f} %)")
    by = collections.defaultdict(lambda: [0, 0])
    for s, e, n in win:
        by[n][0] += 1
        by[n][1] += e - s
    print("top kernels (per step: launches, summed us, mean us):")
    for n, (c, t) in sorted(by.items(), key=lambda x: -x[1][1])[:25]:
        print(f"  {c / nsteps:5.1f} {t / 1e3 / nsteps:8.1f} {t / c / 1e3:7.2f}  {n[:110]}")


if __name__ == "__main__":
    main()
