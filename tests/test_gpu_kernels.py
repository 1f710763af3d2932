"""Per-kernel GPU checks through the C ABI: every GEMM variant against a float64
numpy reference on the same fp16 inputs (fp32 accumulation: |err| ~ 1e-3 relative)."""
import numpy as np
import pytest

from open_speech_amd import dims as D
from open_speech_amd.engine import WhisperEngine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    d = D.WhisperDims(n_mels=80, n_audio_state=128, n_audio_head=2, n_audio_layer=1, n_text_state=128,
                      n_text_head=2, n_text_layer=1)
    e = WhisperEngine(d, device=0, max_batch=1)
    yield e
    e.close()


@pytest.mark.parametrize("variant,M,N,K", [
    (1, 300, 200, 128), (1, 1500, 1280, 1280), (2, 1000, 700, 192), (2, 2048, 1280, 640), (4, 1000, 700, 192),
    (4, 2048, 1280, 640), (4, 700, 300, 64), (4, 513, 1000, 128), (4, 3000, 2304, 1280), (2, 777, 264, 128),
    (3, 1, 1280, 1280), (3, 7, 51866, 384), (3, 64, 5120, 1280), (3, 33, 1280, 5120), (0, 5, 300, 256),
    (3, 64, 51866, 1280), (3, 16, 384, 1536), (3, 3, 700, 128), (3, 50, 40000, 640),
    (5, 64, 51866, 1280), (5, 1, 51866, 1280), (5, 37, 20000, 384), (5, 64, 300, 64), (5, 5, 1000, 128),
    (6, 1500, 1280, 1280), (6, 300, 200, 128), (6, 1500, 5120, 1280), (6, 1500, 1280, 5120),
    (7, 1500, 1280, 1280), (7, 300, 200, 128), (11, 1500, 1280, 1280), (11, 300, 200, 128),
    (11, 1500, 5120, 1280), (11, 1500, 1280, 5120), (11, 6000, 3840, 1280), (11, 2999, 776, 192),
    (16, 1500, 3840, 1280), (16, 1500, 1280, 5120), (16, 700, 264, 128), (16, 513, 1000, 64), (16, 6000, 1280, 1280),
    (16, 257, 136, 192)])
def test_gemm_variants(eng, variant, M, N, K):
    rng = np.random.default_rng(M * 7 + N)
    A = rng.uniform(-1, 1, (M, K)).astype(np.float16)
    W = rng.uniform(-1, 1, (N, K)).astype(np.float16)
    C, ms = eng.debug_gemm(A, W, variant)
    ref = A.astype(np.float64) @ W.astype(np.float64).T
    err = np.abs(C - ref)
    assert err.max() < 2e-3 * np.sqrt(K), (err.max(), ms)


@pytest.mark.parametrize("M,N,K", [(1500, 1280, 1280), (3000, 2304, 1280), (1500, 1280, 5120), (777, 264, 128)])
def test_tile_sizes_bit_identical(eng, M, N, K):
    """The encoder GEMM picks its tile by M (64 for one or a few windows, with or without
    the deep LDS ring, 128 with or without the 4-slot ring, the half-width 256 x 128
    8-wave tile, or the 8-phase 256 at large M): every output element is the same MFMA
    chain over K in the same order, so a window's encoder output does not depend on its batch."""
    rng = np.random.default_rng(M + N + K)
    A = rng.uniform(-1, 1, (M, K)).astype(np.float16)
    W = rng.uniform(-1, 1, (N, K)).astype(np.float16)
    c1, _ = eng.debug_gemm(A, W, 1)
    c6, _ = eng.debug_gemm(A, W, 6)
    c7, _ = eng.debug_gemm(A, W, 7)
    c4, _ = eng.debug_gemm(A, W, 4)
    c11, _ = eng.debug_gemm(A, W, 11)
    c16, _ = eng.debug_gemm(A, W, 16)
    assert np.array_equal(c1, c11)
    assert np.array_equal(c1, c16)
    assert np.array_equal(c1, c6)
    assert np.array_equal(c1, c7)
    assert np.array_equal(c1, c4)


@pytest.mark.parametrize("M,N,K", [(2048, 1280, 1280), (1000, 776, 192)])
def test_8phase_transposed_epilogues_bit_identical(eng, M, N, K):
    """The 8-phase GEMM's fp16 epilogues run on transposed accumulators (Cᵀ = W·Aᵀ: the
    same products in the same K order): debug variants 8 / 10 (fp16, fp16 +
    GELU, transposed) equal 12 / 13 (the same epilogues on the plain accumulators) bit for
    bit, and the fp16 values match float64 references."""
    rng = np.random.default_rng(M * 3 + N + K)
    A = rng.uniform(-1, 1, (M, K)).astype(np.float16)
    W = rng.uniform(-1, 1, (N, K)).astype(np.float16)

    def f16(C):  # the fp16 epilogues write an [M][N] fp16 matrix at the start of the buffer
        return np.ascontiguousarray(C).view(np.uint16).ravel()[:M * N].copy()

    c8, c12 = f16(eng.debug_gemm(A, W, 8)[0]), f16(eng.debug_gemm(A, W, 12)[0])
    c10, c13 = f16(eng.debug_gemm(A, W, 10)[0]), f16(eng.debug_gemm(A, W, 13)[0])
    c18, c19 = f16(eng.debug_gemm(A, W, 18)[0]), f16(eng.debug_gemm(A, W, 19)[0])  # the half-width tile
    assert np.array_equal(c8, c12)
    assert np.array_equal(c10, c13)
    assert np.array_equal(c8, c18)
    assert np.array_equal(c10, c19)
    ref = A.astype(np.float64) @ W.astype(np.float64).T
    from scipy.special import erf
    gelu = 0.5 * ref * (1.0 + erf(ref / np.sqrt(2.0)))
    out = c8.view(np.float16).reshape(M, N).astype(np.float64)
    outg = c10.view(np.float16).reshape(M, N).astype(np.float64)
    tol = 2e-3 * np.sqrt(K)
    assert np.abs(out - ref).max() < tol + 1e-3 * np.abs(ref).max()
    assert np.abs(outg - gelu).max() < tol + 1e-3 * np.abs(gelu).max()
