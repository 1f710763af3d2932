// MFMA GEMM for gfx950:  C[M,N] = A[M,K] · W[N,K]ᵀ (+ bias, fused epilogue).
//
// Every dense layer of Whisper (conv stem as implicit GEMM, q/k/v, out-proj, MLP,
// cross-attention K/V precompute, logits) goes through this one kernel family.
// Tile 128x128x64, 4 waves (2x2, 64x64 per wave = 4x4 v_mfma_f32_16x16x32_f16),
// fp16 operands, fp32 accumulation.  Operand tiles are staged global->LDS with
// 16-byte global_load_lds (no VGPR round trip), double buffered; the LDS image is
// XOR-swizzled on the 16-B chunk (chunk ^ ((row>>1)&7)) through the per-lane
// SOURCE address so the ds_read_b128 fragment reads are conflict-free
// (cdna_hip_programming.md §5 rule 21, T2).
//
// A rows may be "grouped": row m lives at A + (m / a_grp_rows)*a_grp_stride +
// (m % a_grp_rows)*lda.  That lets the conv stem read an overlapping 3-row window
// of a time-major activation as one GEMM row (lda = C or 2C, K = 3C) without an
// im2col copy, and lets a batch of windows with padded per-window buffers be one
// GEMM.  The C side has the same addressing.
#include "common.h"

namespace osw {

namespace {
constexpr int BM = 128, BN = 128, BK = 64, NTHR = 256;

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

__device__ __forceinline__ const h16* grp_row(const h16* base, int64_t m, int64_t grp_rows, int64_t grp_stride,
                                              int64_t ld) {
    return base + (m / grp_rows) * grp_stride + (m % grp_rows) * ld;
}

template <int EPI>
__device__ __forceinline__ void store_one(const GemmArgs& g, int m, int n, float v) {
    if (g.bias) v += g.bias[n];
    const int64_t grp = m / g.c_grp_rows, r = m % g.c_grp_rows;
    if constexpr (EPI == EPI_F16 || EPI == EPI_F16_GELU) {
        if (EPI == EPI_F16_GELU) v = gelu_erf(v);
        h16* C = (h16*)g.C + grp * g.c_grp_stride + r * g.ldc;
        C[n] = (h16)v;
    } else if constexpr (EPI == EPI_F32_RESID) {
        float* C = (float*)g.C + grp * g.c_grp_stride + r * g.ldc;
        C[n] += v;
    } else if constexpr (EPI == EPI_F32_GELU_POS) {
        float* C = (float*)g.C + grp * g.c_grp_stride + r * g.ldc;
        C[n] = gelu_erf(v) + g.pos[r * (int64_t)g.N + n];
    } else if constexpr (EPI == EPI_F32) {
        float* C = (float*)g.C + grp * g.c_grp_stride + r * g.ldc;
        C[n] = v;
    } else {  // EPI_HEADS: n = which*D + h*64 + d ; m = b*T + t
        const int D = g.heads_H * 64;
        const int which = n / D, h = (n % D) >> 6, d = n & 63;
        const int b = m / g.heads_T, t = m % g.heads_T;
        h16* C = (h16*)g.C;
        C[((((int64_t)which * g.heads_nb + b) * g.heads_H + h) * g.heads_T + t) * 64 + d] = (h16)v;
    }
}

template <int EPI>
__global__ __launch_bounds__(NTHR, 2) void gemm_kernel(GemmArgs g) {
    __shared__ __attribute__((aligned(16))) h16 lds[2][2][BM * BK];  // [buf][A|W], 64 KiB
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;

    // per-thread source rows for the 4 A and 4 W glds pieces (fixed over K)
    const h16* asrc[4];
    const h16* wsrc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = (i * 4 + wave) * 8 + (lane >> 3);
        const int c = swz(r, lane & 7);
        const int gm = min(m0 + r, g.M - 1);
        const int gn = min(n0 + r, g.N - 1);
        asrc[i] = grp_row(g.A, gm, g.a_grp_rows, g.a_grp_stride, g.lda) + c * 8;
        wsrc[i] = g.W + (int64_t)gn * g.ldw + c * 8;
    }

    auto stage = [&](int buf, int k0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            h16* da = &lds[buf][0][(i * 4 + wave) * 8 * BK];
            h16* dw = &lds[buf][1][(i * 4 + wave) * 8 * BK];
            __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + k0), (OSW_LDS void*)da, 16, 0, 0);
            __builtin_amdgcn_global_load_lds((const void*)(wsrc[i] + k0), (OSW_LDS void*)dw, 16, 0, 0);
        }
    };

    const int wm = wave >> 1, wn = wave & 1;
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = g.K / BK;
    stage(0, 0);
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) & lgkmcnt(0)
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) stage(buf ^ 1, (kt + 1) * BK);
        const h16* la = lds[buf][0];
        const h16* lw = lds[buf][1];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int c = ks * 4 + (lane >> 4);
            h16x8 a[4], b[4];
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) {
                const int row = wm * 64 + mi * 16 + (lane & 15);
                a[mi] = *(const h16x8*)&la[row * BK + swz(row, c) * 8];
            }
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) {
                const int row = wn * 64 + ni * 16 + (lane & 15);
                b[ni] = *(const h16x8*)&lw[row * BK + swz(row, c) * 8];
            }
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int ni = 0; ni < 4; ++ni)
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
        }
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
    }

#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = m0 + wm * 64 + mi * 16 + (lane >> 4) * 4 + i;
            if (m >= g.M) continue;
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) {
                const int n = n0 + wn * 64 + ni * 16 + (lane & 15);
                if (n < g.N) store_one<EPI>(g, m, n, acc[mi][ni][i]);
            }
        }
}
// ---------------------------------------------------------------------------
// Skinny GEMM for the decoder (M <= 64 rows = windows in the batch): weight-
// bandwidth bound, so the grid is split over N (64 columns per workgroup, 16 per
// wave) AND over K (ksplit partial slabs, reduced deterministically by a second
// kernel that also applies the epilogue).  Operands go straight to VGPRs
// (no LDS: nothing is shared between waves but the tiny, L2-resident A).
template <int MT, bool DIRECT, int EPI>
__global__ __launch_bounds__(256) void gemm_skinny_kernel(GemmArgs g, int kc, float* __restrict__ part) {
    constexpr int U = 4;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nb = blockIdx.x * 64 + wave * 16;
    const int ks = blockIdx.y;
    const int k0 = ks * kc;
    const int n = min(nb + (lane & 15), g.N - 1);
    const h16* wrow = g.W + (int64_t)n * g.ldw + k0 + 8 * (lane >> 4);
    const h16* arow[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int m = min(mt * 16 + (lane & 15), g.M - 1);
        arow[mt] = grp_row(g.A, m, g.a_grp_rows, g.a_grp_stride, g.lda) + k0 + 8 * (lane >> 4);
    }
    f32x4 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < kc; k += 32 * U) {
        h16x8 wf[U];
#pragma unroll
        for (int u = 0; u < U; ++u) wf[u] = *(const h16x8*)(wrow + k + 32 * u);
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                const h16x8 af = *(const h16x8*)(arow[mt] + k + 32 * u);
                acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, wf[u], acc[mt], 0, 0, 0);
            }
        }
    }
    const int col = nb + (lane & 15);
    if (col >= g.N) return;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = mt * 16 + (lane >> 4) * 4 + i;
            if (m >= g.M) continue;
            if constexpr (DIRECT) store_one<EPI>(g, m, col, acc[mt][i]);
            else part[((int64_t)ks * g.M + m) * g.N + col] = acc[mt][i];
        }
}

template <int EPI>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmArgs g, int ksplit, const float* __restrict__ part) {
    const int64_t total = (int64_t)g.M * g.N;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        float v = 0.f;
        for (int s = 0; s < ksplit; ++s) v += part[s * total + i];
        store_one<EPI>(g, (int)(i / g.N), (int)(i % g.N), v);
    }
}

template <int MT, int EPI>
void skinny_dispatch(const GemmArgs& g, int ksplit, float* part, hipStream_t s) {
    const dim3 grid((g.N + 63) / 64, ksplit);
    const int kc = g.K / ksplit;
    if (ksplit == 1) {
        gemm_skinny_kernel<MT, true, EPI><<<grid, 256, 0, s>>>(g, kc, part);
    } else {
        gemm_skinny_kernel<MT, false, EPI><<<grid, 256, 0, s>>>(g, kc, part);
        const int64_t total = (int64_t)g.M * g.N;
        splitk_reduce_kernel<EPI><<<(unsigned)std::min<int64_t>((total + 255) / 256, 1024), 256, 0, s>>>(g, ksplit, part);
    }
}

template <int EPI>
void skinny_mt(const GemmArgs& g, int ksplit, float* part, hipStream_t s) {
    switch ((g.M + 15) / 16) {
        case 1: skinny_dispatch<1, EPI>(g, ksplit, part, s); break;
        case 2: skinny_dispatch<2, EPI>(g, ksplit, part, s); break;
        case 3: skinny_dispatch<3, EPI>(g, ksplit, part, s); break;
        default: skinny_dispatch<4, EPI>(g, ksplit, part, s); break;
    }
}
}  // namespace

// split count: a divisor of K/128 giving 256..1024 workgroups when possible
int skinny_ksplit(int N, int K) {
    const int nbn = (N + 63) / 64;
    const int kt = K / 128;
    int best = 1;
    for (int d = 1; d <= kt; ++d) {
        if (kt % d) continue;
        if ((int64_t)nbn * d > 1024) break;
        best = d;
        if ((int64_t)nbn * d >= 256) break;
    }
    return best;
}

void launch_gemm_skinny(const GemmArgs& g, float* part, hipStream_t s) {
    const int ks = skinny_ksplit(g.N, g.K);
    switch (g.epi) {
        case EPI_F16: skinny_mt<EPI_F16>(g, ks, part, s); break;
        case EPI_F16_GELU: skinny_mt<EPI_F16_GELU>(g, ks, part, s); break;
        case EPI_F32_RESID: skinny_mt<EPI_F32_RESID>(g, ks, part, s); break;
        case EPI_F32: skinny_mt<EPI_F32>(g, ks, part, s); break;
        default: break;  // other epilogues are encoder-only
    }
}

void launch_gemm(const GemmArgs& g, hipStream_t s) {
    dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM);
    switch (g.epi) {
        case EPI_F16: gemm_kernel<EPI_F16><<<grid, NTHR, 0, s>>>(g); break;
        case EPI_F16_GELU: gemm_kernel<EPI_F16_GELU><<<grid, NTHR, 0, s>>>(g); break;
        case EPI_F32_RESID: gemm_kernel<EPI_F32_RESID><<<grid, NTHR, 0, s>>>(g); break;
        case EPI_F32_GELU_POS: gemm_kernel<EPI_F32_GELU_POS><<<grid, NTHR, 0, s>>>(g); break;
        case EPI_F32: gemm_kernel<EPI_F32><<<grid, NTHR, 0, s>>>(g); break;
        default: gemm_kernel<EPI_HEADS><<<grid, NTHR, 0, s>>>(g); break;
    }
}

}  // namespace osw
