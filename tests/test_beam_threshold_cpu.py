"""The beam select's threshold form of the per-slice top-2K (decode.hip, beam_slice_body
FAST) restated on the CPU against the pop form it replaced, on crafted slices: coarse
quantised logits (many ties at the cutoff), +/-inf and NaN entries, masks of every density,
ragged slice ends.  Both restatements follow the kernel's thread map (256 threads = 4 waves
x 64 lanes, entry u of thread t is token lo + 256 u + t) and order (key desc, token asc).
The candidate lists feed beam_update, whose ranking is pinned to the oracle's CTranslate2
BeamSearch restatement by the GPU beam tests; this test pins that the threshold form picks
exactly the lists the pops picked, including the cases where it must fall back to them.
"""
import numpy as np
import pytest

VPT, NT, SCAP = 16, 256, 256
INT_MAX = 2**31 - 1


def _entries(x, ok, lo, hi):
    """(key, token, live) per (u, t): the kernel's xv / okA / live bits."""
    u = np.arange(VPT)[:, None]
    t = np.arange(NT)[None, :]
    tok = lo + u * 256 + t
    valid = tok < hi
    xv = np.where(valid, x[np.minimum(tok, hi - 1) - lo], np.nan)
    live = valid & ~np.isnan(xv)
    allowed = valid & ok[np.minimum(tok, hi - 1) - lo]
    key = np.where(allowed, xv, -np.inf)
    return xv, key, tok, live, allowed


def pops(x, ok, lo, hi, k2):
    """decode.hip beam_slice_body `pops`: K2 times the best unused live entry."""
    _, key, tok, live, _ = _entries(x, ok, lo, hi)
    cand = sorted(((-float(key[i]), int(tok[i])) for i in zip(*np.nonzero(live))))
    out = [(-s, i) for s, i in cand[:k2]]
    return out + [(-np.inf, INT_MAX)] * (k2 - len(out))


def fast(x, ok, lo, hi, k2):
    """beam_slice_body FAST: None where the kernel falls back to the pops."""
    xv, _, tok, live, allowed = _entries(x, ok, lo, hi)
    al = allowed & live
    lm = np.where(al, xv, -np.inf).max(axis=0)  # lane maxima, per thread
    tw = []
    for w in range(4):
        c = lm[64 * w:64 * (w + 1)].copy()
        t = np.inf
        for _ in range(k2):  # wave pops: argmax, ties to the lower lane
            j = int(np.argmax(c))
            t = c[j]
            c[j] = -np.inf
        tw.append(t)
    T = max(tw)
    if T == -np.inf:
        return None
    sel = al & (xv >= T)
    if sel.sum() > SCAP:
        return None
    S = sorted((-float(xv[i]), int(tok[i])) for i in zip(*np.nonzero(sel)))
    assert len(S) >= k2  # the guarantee the kernel relies on
    return [(-s, i) for s, i in S[:k2]]


def _case(rng, kind):
    V = 51866
    per = (V + 15) // 16
    sl = int(rng.integers(0, 16))
    lo, hi = sl * per, min(V, sl * per + per)
    n = hi - lo
    if kind == "gauss":
        x = rng.normal(0, 3, n).astype(np.float32)
    elif kind == "coarse":  # ties everywhere, also at the cutoff
        x = np.round(rng.normal(0, 1, n) * 2).astype(np.float32)
    elif kind == "few_levels":
        x = rng.choice(np.float32([-1.0, 0.0, 2.5, 2.5, 7.0]), n)
    else:  # "specials"
        x = rng.normal(0, 2, n).astype(np.float32)
        for val, frac in ((np.inf, 0.0005), (-np.inf, 0.2), (np.nan, 0.05)):
            x[rng.random(n) < frac] = val
    density = float(rng.choice([1.0, 0.5, 0.05, 0.004, 0.0008]))
    ok = rng.random(n) < density
    return x, ok, lo, hi


@pytest.mark.parametrize("kind", ["gauss", "coarse", "few_levels", "specials"])
def test_threshold_lists_equal_pops(kind):
    rng = np.random.default_rng({"gauss": 1, "coarse": 2, "few_levels": 3, "specials": 4}[kind])
    fell_back = used = 0
    for _ in range(60):
        x, ok, lo, hi = _case(rng, kind)
        k2 = 2 * int(rng.choice([2, 5, 8]))
        ref = pops(x, ok, lo, hi, k2)
        got = fast(x, ok, lo, hi, k2)
        if got is None:
            fell_back += 1
            continue
        used += 1
        assert got == ref
    assert used > 0
    if kind == "few_levels":
        assert fell_back > 0  # > 256 entries tie at the threshold: the pops take over
