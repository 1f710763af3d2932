"""The GEMM epilogues' fast_div (open-speech_amd/csrc/gemm.hip): m / d by a float
reciprocal and one correction step, claimed exact for 0 <= m < 2^22.  Restated in
float32 numpy with the reciprocal rounded to nearest and one ulp either way (v_rcp_f32
is accurate to 1 ulp), over every divisor the encoder uses and a spread of others, at
the multiples of d and their neighbours (where truncation can land one off) up to 2^22."""
import numpy as np


def fast_div(m, d, rcp):
    q = np.trunc(m.astype(np.float32) * rcp).astype(np.int64)
    r = m - q * d
    return q + (r >= d) - (r < 0)


def test_fast_div_exact_below_2_22():
    lim = 1 << 22
    divisors = [1, 2, 3, 7, 64, 448, 1280, 1500, 2560, 3000, 3840, 5120, 6000, 96000] + \
        list(range(5, 5000, 97)) + [lim - 1]
    for d in divisors:
        k = np.arange(0, lim // d + 1, max(1, (lim // d) // 4096), dtype=np.int64)
        m = np.concatenate([k * d - 1, k * d, k * d + 1, np.arange(0, min(lim, 4096), dtype=np.int64)])
        m = m[(m >= 0) & (m < lim)]
        r0 = np.float32(1.0) / np.float32(d)
        for rcp in (np.nextafter(r0, np.float32(0)), r0, np.nextafter(r0, np.float32(1))):
            q = fast_div(m, d, rcp)
            assert np.array_equal(q, m // d), d
