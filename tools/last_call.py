#!/usr/bin/env python3
"""Per-kernel table of the last engine call in a rocprofv3 kernel_trace.csv (cut at the
last log-mel launch), plus its wall span.  usage: last_call.py run_kernel_trace.csv"""
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from trace_summary import table  # noqa: E402

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
mel = [i for i, r in enumerate(rows) if "mel_logmel_kernel" in r["Kernel_Name"]]
seg = rows[mel[-1]:]
print(table(seg, "# last call"))
print("wall span ms", (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e6)
