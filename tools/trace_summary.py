#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_trace.csv of `bench.py`: per-kernel totals over the
whole run, and the same for the isolated roofline pass alone (the 64-clip step lane 0
runs after the timed region, where the bench's `roofline.avg_launch_ms` comes from)
and for the isolated beam-5 step after it.  After the timed region the bench runs:
roofline pass, beam-5 step (unless --beam5 0), R latency repeats (--latency-repeats),
one log-mel launch each, so the passes are cut at the trailing log-mel launches.

usage: trace_summary.py run_kernel_trace.csv out_prefix [latency_repeats] [beam5]
writes out_prefix_kernel_summary.txt, out_prefix_roofline_pass.txt and (beam5 = 1,
the default) out_prefix_beam5_pass.txt"""
import csv
import sys
from collections import defaultdict


def table(rows, title):
    agg = defaultdict(lambda: [0, 0])
    for r in rows:
        a = agg[r["Kernel_Name"]]
        a[0] += 1
        a[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot = sum(a[1] for a in agg.values()) or 1
    out = [title]
    for name, (n, ns) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        out.append(f"{ns / 1e6:9.2f} ms {100 * ns / tot:6.2f}% n={n:>6} avg={ns / n / 1e3:9.2f}us {name[:110]}")
    out.append(f"total kernel time {tot / 1e6:.2f} ms over {sum(a[0] for a in agg.values())} dispatches")
    return "\n".join(out) + "\n"


def main():
    path, prefix = sys.argv[1], sys.argv[2]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    beam5 = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    with open(prefix + "_kernel_summary.txt", "w") as fh:
        fh.write(table(rows, f"# all kernels of the run ({path})"))
    mel = [i for i, r in enumerate(rows) if "mel_logmel_kernel" in r["Kernel_Name"]]
    tail = reps + beam5
    if len(mel) < tail + 1:
        return
    cut = lambda k: mel[-k] if k else len(rows)  # start of the k-th last pass
    with open(prefix + "_roofline_pass.txt", "w") as fh:
        fh.write(table(rows[cut(tail + 1):cut(tail)], "# isolated roofline pass (1 lane, eager decode, 64 clips)"))
    if beam5:
        with open(prefix + "_beam5_pass.txt", "w") as fh:
            fh.write(table(rows[cut(reps + 1):cut(reps)], "# isolated beam-5 step (1 lane, 64 clips)"))


if __name__ == "__main__":
    main()
