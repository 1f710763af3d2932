#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (<name>_results.db, the default output format of
ROCm 7 rocprofv3 --kernel-trace): top kernels by total time, in the same format as
kstats.py.  Optional second argument: also write a kernel_stats-style CSV there.

usage: kstats_db.py run_results.db [out.csv] [--gaps] [top_n]
--gaps: also print the busy time vs. wall span of the kernel stream and the idle gap
before each kernel class (launch boundaries; the stream is assumed to be serial).
"""
import csv
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
out_csv = sys.argv[2] if len(sys.argv) > 2 and sys.argv[2].endswith(".csv") else None
n = int(sys.argv[-1]) if sys.argv[-1].isdigit() else 30
gaps = "--gaps" in sys.argv
c = sqlite3.connect(db)
agg = defaultdict(lambda: [0, 0.0, float("inf"), 0.0])
for name, dur in c.execute("select name, duration from kernels"):
    a = agg[name]
    a[0] += 1
    a[1] += dur
    a[2] = min(a[2], dur)
    a[3] = max(a[3], dur)
tot = sum(a[1] for a in agg.values())
rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
for name, (calls, s, mn, mx) in rows[:n]:
    print(f"{s / 1e6:9.2f} ms {100 * s / tot:6.2f}% n={calls:>6} avg={s / calls / 1e3:9.2f}us {name[:100]}")
print(f"total kernel time {tot / 1e6:.2f} ms")
if out_csv:
    with open(out_csv, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, (calls, s, mn, mx) in rows:
            w.writerow([name, calls, int(s), s / calls, 100 * s / tot, int(mn), int(mx)])
if gaps:
    ev = sorted(c.execute("select name, start, end from kernels"), key=lambda r: r[1])
    busy = sum(e - s for _, s, e in ev)
    gap_by = defaultdict(lambda: [0, 0.0])
    big = 0.0
    for (n0, s0, e0), (n1, s1, e1) in zip(ev, ev[1:]):
        g = s1 - e0
        if g > 200e3:  # > 200 us: host-side pause (sync, python), not a launch boundary
            big += g
            continue
        gap_by[n1][0] += 1
        gap_by[n1][1] += max(0, g)
    span = ev[-1][2] - ev[0][1]
    small = sum(v[1] for v in gap_by.values())
    print(f"kernels {len(ev)}: busy {busy / 1e6:.2f} ms, span {span / 1e6:.2f} ms, "
          f"boundary gaps {small / 1e6:.2f} ms ({small / max(1, len(ev)) / 1e3:.2f} us avg), host pauses {big / 1e6:.2f} ms")
    for name, (k, g) in sorted(gap_by.items(), key=lambda kv: -kv[1][1])[:12]:
        print(f"  gap before {name[:80]}: n={k} avg {g / k / 1e3:.2f} us")
