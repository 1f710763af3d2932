#!/usr/bin/env python3
"""Lane timeline of a rocprofv3 kernel trace of bench.py's lanes (tools/gpu_trace.sh):
per stream, the encoder phases (mel .. cross-K/V GEMM) and, for every window of time
cut at encoder starts/ends, how many decoder steps each lane completed (4 cross-
attention launches = one step) and the per-kernel mean durations of one lane in a
window where another lane encodes vs where none does.

usage: lane_timeline.py run_kernel_trace.csv[.gz] [out.txt]"""
import collections
import csv
import gzip
import sys

ENC = ("gemm8p", "enc_attn", "layernorm_kernel", "mel_", "gemm_kernel", "gemm64_ring")


def load(path):
    fh = gzip.open(path, "rt") if path.endswith(".gz") else open(path)
    rows = sorted(csv.DictReader(fh), key=lambda r: int(r["Start_Timestamp"]))
    t0 = int(rows[0]["Start_Timestamp"])
    out = []
    for r in rows:
        out.append(((int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - t0) / 1e6, r["Stream_Id"],
                    r["Kernel_Name"], r["Grid_Size_X"] + "x" + r["Grid_Size_Y"]))
    return out


def main():
    ev = load(sys.argv[1])
    out = open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout
    lanes = sorted({st for _, _, st, n, _ in ev if "dec_xattn" in n})
    # encoder phases: from a mel_window launch to the last encoder-class kernel before the next decoder kernel
    phases = collections.defaultdict(list)
    for st in lanes:
        cur = None
        for s, e, s2, n, _ in ev:
            if s2 != st:
                continue
            if "mel_window" in n:
                cur = [s, e]
            elif cur is not None and any(k in n for k in ENC):
                cur[1] = e
            elif cur is not None:
                phases[st].append(tuple(cur))
                cur = None
        if cur:
            phases[st].append(tuple(cur))
        print(f"lane(stream {st}) encoder phases (ms): " + " ".join(f"[{a:.0f},{b:.0f}]" for a, b in phases[st]), file=out)
    cuts = sorted({t for st in lanes for ph in phases[st] for t in ph})
    print("\nwindow            encoding-lanes  decoder steps per lane", file=out)
    for a, b in zip(cuts, cuts[1:]):
        if b - a < 5:
            continue
        enc = [st for st in lanes if any(p0 <= a and b <= p1 + 1e-6 for p0, p1 in phases[st])]
        steps = {st: sum(1 for s, _, s2, n, _ in ev if s2 == st and "dec_xattn" in n and a <= s < b) / 4 for st in lanes}
        print(f"[{a:7.0f},{b:7.0f}] {','.join(enc) or '-':>14}  " +
              "  ".join(f"{st}:{steps[st]:6.1f}" for st in lanes) + f"   ({(b - a):.0f} ms)", file=out)
    # per-kernel means for one decoding lane: while another lane encodes vs while none does
    agg = {True: collections.defaultdict(lambda: [0, 0.0]), False: collections.defaultdict(lambda: [0, 0.0])}
    for st in lanes:
        for s, e, s2, n, g in ev:
            if s2 != st or any(k in n for k in ENC) or "rocclr" in n:
                continue
            if any(p0 <= s <= p1 for p0, p1 in phases[st]):
                continue
            other = any(p0 <= s <= p1 for o in lanes if o != st for p0, p1 in phases[o])
            k = n.split("(")[0][-48:] + " " + g
            agg[other][k][0] += 1
            agg[other][k][1] += e - s
    for other in (True, False):
        print(f"\ndecoder kernels of a lane while {'another lane encodes' if other else 'no lane encodes'}:", file=out)
        for k, (c, t) in sorted(agg[other].items(), key=lambda kv: -kv[1][1])[:14]:
            print(f"  {k:72s} n={c:6d} mean={1e3 * t / c:8.1f} us  total={t:8.1f} ms", file=out)


if __name__ == "__main__":
    main()
