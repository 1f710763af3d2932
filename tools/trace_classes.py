#!/usr/bin/env python3
"""Kernel-trace summary by class for a serving-style run (config 5, REST probes):
total and mean time per kernel class (encoder GEMM / attention / LayerNorm, decoder
projections, residual+LN, attentions, selection, ...), per-kernel top list, and the
union of all kernel intervals against the traced span, i.e. how much of the wall
time the GPU ran nothing (host and launch overhead).

usage: trace_classes.py run_kernel_trace.csv [out.txt]"""
import csv
import sys
from collections import defaultdict

CLASSES = [
    ("enc_gemm", ("gemm8p", "gemm_kernel<", "gemm64_ring", "gemm128_ring")),
    ("enc_attn", ("enc_attn",)),
    ("enc_ln", ("layernorm_kernel",)),
    ("mel", ("mel_",)),
    ("dec_proj", ("gemm_skinny", "gemm_wide", "gemm_tiled")),
    ("dec_resln", ("dec_resid_ln", "dec_reduce")),
    ("dec_self", ("dec_self_attn",)),
    ("dec_cross", ("dec_xattn",)),
    ("select", ("select_kernel", "beam_update", "count_done")),
    ("copy", ("rocclr",)),
]


def cls(name):
    for c, keys in CLASSES:
        if any(k in name for k in keys):
            return c
    return "other"


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    out = open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    if not iv:
        print("empty trace", file=out)
        return
    span = iv[-1][1] - iv[0][0]
    union, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e, _ in iv[1:]:
        if s > ce:
            union += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    union += ce - cs
    agg = defaultdict(lambda: [0, 0])
    per = defaultdict(lambda: [0, 0])
    for s, e, n in iv:
        a = agg[cls(n)]
        a[0] += 1
        a[1] += e - s
        p = per[n]
        p[0] += 1
        p[1] += e - s
    tot = sum(a[1] for a in agg.values())
    print(f"span {span / 1e6:.1f} ms, GPU busy (union of kernels) {union / 1e6:.1f} ms = {100 * union / span:.1f} %, "
          f"kernel time (sum) {tot / 1e6:.1f} ms, {len(iv)} dispatches", file=out)
    for c, (n, ns) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{c:10s} {ns / 1e6:9.2f} ms {100 * ns / tot:6.2f}% n={n:>8} avg={ns / n / 1e3:8.2f}us", file=out)
    print("", file=out)
    for name, (n, ns) in sorted(per.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f"{ns / 1e6:9.2f} ms {100 * ns / tot:6.2f}% n={n:>8} avg={ns / n / 1e3:8.2f}us {name[:110]}", file=out)


if __name__ == "__main__":
    main()
