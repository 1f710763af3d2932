#!/usr/bin/env python3
"""One decode step's kernel timeline from a rocprofv3 kernel trace: the kernels between the
N-th and (N+1)-th launch of a marker kernel (default: the beam update), with each one's start
relative to the first, its duration, and the gap since the previous kernel ended.
usage: step_timeline.py run_kernel_trace.csv [marker_substring] [occurrence]"""
import csv
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "beam_update"
occ = int(sys.argv[3]) if len(sys.argv) > 3 else 200
rows = []
for r in csv.DictReader(open(path)):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:80], r.get("Queue_Id", "")))
rows.sort()
idx = [i for i, r in enumerate(rows) if marker in r[2]]
if len(idx) <= occ + 1:
    occ = max(0, len(idx) - 2)
a, b = idx[occ], idx[occ + 1]
t0 = rows[a + 1][0]
prev_end = rows[a][1]
tot = 0.0
for s, e, name, q in rows[a + 1:b + 1]:
    print(f"{(s - t0) / 1e3:8.2f} us  dur {(e - s) / 1e3:7.2f}  gap {(s - prev_end) / 1e3:6.2f}  q{q}  {name}")
    prev_end = e
    tot += (e - s) / 1e3
print(f"step span {(rows[b][1] - t0) / 1e3:.1f} us, kernel time {tot:.1f} us")
