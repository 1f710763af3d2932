#!/usr/bin/env python3
"""Per-dispatch values of one counter, in dispatch order, for the kernels whose name
contains a substring (rocprofv3 --pmc counter_collection.csv).  FETCH_SIZE is doubled
(gfx950 correction, MI355X_MICROARCH.md HBM section) and printed in MB.
usage: pmc_dispatch.py file.csv COUNTER SUBSTRING"""
import csv
import sys

path, counter, sub = sys.argv[1], sys.argv[2], sys.argv[3]
rows = []
for r in csv.DictReader(open(path)):
    if r.get("Counter_Name") != counter or sub not in r["Kernel_Name"]:
        continue
    rows.append((int(r.get("Dispatch_Id", len(rows))), r["Kernel_Name"], float(r["Counter_Value"])))
rows.sort()
scale = 2 * 1024 / 1e6 if counter == "FETCH_SIZE" else 1024 / 1e6
for d, k, v in rows:
    print(f"{d:6d}  {v * scale:10.1f} MB  {k[:90]}")
