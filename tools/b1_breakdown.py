#!/usr/bin/env python3
"""Per-step kernel breakdown of the batch-1 greedy decode from a rocprofv3 kernel trace of
`bench.py --lanes 1 --steps 1 --latency-repeats N` (tools/gpu_run.sh b1): kernels grouped by
(name, grid), keeping the groups whose launch count is a multiple of the batch-1 step count
(the 64-window step's launches have other grids), with the mean duration and the launches
per step.  usage: b1_breakdown.py run_kernel_trace.csv[.gz] steps"""
import collections
import csv
import gzip
import sys


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    fh = gzip.open(path, "rt") if path.endswith(".gz") else open(path)
    groups = collections.defaultdict(list)
    for r in csv.DictReader(fh):
        key = (r["Kernel_Name"][:90], r["Grid_Size_X"] + "x" + r["Grid_Size_Y"] + "x" + r["Grid_Size_Z"])
        groups[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = []
    for (name, grid), d in groups.items():
        if len(d) < steps:
            continue
        per = len(d) / steps
        rows.append((per * sum(d) / len(d), per, sum(d) / len(d), name, grid))
    rows.sort(reverse=True)
    tot = 0.0
    for us_step, per, mean, name, grid in rows:
        tot += us_step
        print(f"{us_step:8.1f} us/step  {per:6.2f}/step  mean {mean:7.2f} us  {grid:>16}  {name}")
    print(f"total {tot:.1f} us per step (groups with >= {steps} launches)")


main()
