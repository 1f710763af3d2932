"""Sampling at temperature > 0 (oracle side): the counter-hash Gumbel-max draw that the
HIP select kernel uses is reproducible and samples softmax(x / T) over the kept tokens."""
import numpy as np

from oracle import decode as odec


def test_gumbel_noise_reproducible_and_keyed():
    v = np.arange(1000)
    a = odec.gumbel_noise(7, 3, 11, v)
    assert a.dtype == np.float32 and np.isfinite(a).all()
    np.testing.assert_array_equal(a, odec.gumbel_noise(7, 3, 11, v))
    for other in (odec.gumbel_noise(8, 3, 11, v), odec.gumbel_noise(7, 4, 11, v), odec.gumbel_noise(7, 3, 12, v)):
        assert np.mean(a == other) < 0.01
    # Gumbel(0, 1): mean = Euler-Mascheroni constant, variance = pi^2 / 6
    g = odec.gumbel_noise(1, 0, 0, np.arange(200000))
    assert abs(float(g.mean()) - 0.5772) < 0.01
    assert abs(float(g.var()) - np.pi ** 2 / 6) < 0.03


def test_sample_token_follows_tempered_softmax():
    x = np.array([1.0, 0.0, -1.0, 2.0, -np.inf, 0.5])
    T = 0.7
    n = 20000
    counts = np.zeros(x.size)
    for seed in range(n):
        counts[odec.sample_token(x, 1.0 / T, seed, 0, 5)] += 1
    keep = np.isfinite(x)
    p = np.exp(x[keep] / T - np.max(x[keep] / T))
    p /= p.sum()
    assert counts[~keep].sum() == 0
    np.testing.assert_allclose(counts[keep] / n, p, atol=0.015)


def test_sample_token_cold_limit_is_argmax():
    rng = np.random.default_rng(0)
    for s in range(50):
        x = rng.standard_normal(300)
        x[rng.integers(0, 300, 40)] = -np.inf
        assert odec.sample_token(x, 1e5, s, 1, 2) == int(np.argmax(x))
