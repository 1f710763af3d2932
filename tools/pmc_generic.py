#!/usr/bin/env python3
"""Mean value per dispatch of every counter in a rocprofv3 counter_collection.csv, per
kernel (top kernels by dispatch count x SQ_WAVE_CYCLES).  usage: pmc_generic.py file.csv"""
import collections
import csv
import sys

per = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    per[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
rows = []
for k, cs in per.items():
    n = max(len(v) for v in cs.values())
    mean = {c: sum(v) / max(1, len(v)) for c, v in cs.items()}
    rows.append((mean.get("SQ_WAVE_CYCLES", 0) * n, k, n, mean))
rows.sort(reverse=True)
for _, k, n, mean in rows[:25]:
    wc = mean.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{k[:100]}\n   n={n} " + " ".join(f"{c}={v:.4g}" for c, v in sorted(mean.items())) +
          f"  | VALU/wave_cyc={mean.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f} wait/wave_cyc={mean.get('SQ_WAIT_ANY', 0) / wc:.3f}")
