#!/usr/bin/env python3
"""Per (kernel, grid, workgroup) launch-time table for one pass of a rocprofv3
kernel_trace.csv of bench.py -- which GEMM shape costs what.  The pass is cut like
trace_summary.py: `pass_from_end` = 0 for the last pass (beam-5 step with
--latency-repeats 0), 1 for the one before it (roofline pass).

usage: trace_shapes.py run_kernel_trace.csv out.txt [pass_from_end] [name_filter]"""
import csv
import sys
from collections import defaultdict


def main():
    path, out = sys.argv[1], sys.argv[2]
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    filt = sys.argv[4] if len(sys.argv) > 4 else ""
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    mel = [i for i, r in enumerate(rows) if "mel_logmel_kernel" in r["Kernel_Name"]]
    lo = mel[-(k + 1)]
    hi = mel[-k] if k else len(rows)
    agg = defaultdict(lambda: [0, 0])
    for r in rows[lo:hi]:
        if filt not in r["Kernel_Name"]:
            continue
        key = (r["Kernel_Name"][:70], r.get("Grid_Size", r.get("Grid_Size_X", "?")),
               r.get("Workgroup_Size", r.get("Workgroup_Size_X", "?")))
        agg[key][0] += 1
        agg[key][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    with open(out, "w") as fh:
        for (name, grid, wg), (n, ns) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            fh.write(f"{ns / 1e6:9.2f} ms n={n:>6} avg={ns / n / 1e3:9.2f}us grid={grid} wg={wg} {name}\n")


if __name__ == "__main__":
    main()
