#!/usr/bin/env python3
"""Summarise a rocprofv3 --stats kernel_stats.csv: top kernels by total time."""
import csv
import sys

r = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(x["TotalDurationNs"]) for x in r)
for x in sorted(r, key=lambda x: -float(x["TotalDurationNs"]))[:n]:
    print(f"{float(x['TotalDurationNs'])/1e6:9.2f} ms {float(x['Percentage']):6.2f}% n={x['Calls']:>6} "
          f"avg={float(x['AverageNs'])/1e3:9.2f}us {x['Name'][:100]}")
print(f"total kernel time {tot/1e6:.2f} ms")
