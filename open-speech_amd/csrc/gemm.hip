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
#include "resln.h"

#include <cstdlib>
#include <mutex>
#include <set>
#include <stdexcept>

namespace osw {

namespace {
#include "select.h"
constexpr int HD = 64;
#include "selfattn.h"

constexpr int BM = 128, BN = 128, BK = 64, NTHR = 256;
#ifndef OSW_SKINNY_CK1
#define OSW_SKINNY_CK1 4  // k32 steps per chunk of the 16-row hi/lo skinny GEMM (A/B builds: 8)
#endif

// Dynamic-LDS limits are set once per kernel, before its first launch, under a lock, and
// all of them when a context is created (prepare_gemm_kernels): a lazily set attribute
// (a racy `static bool` per launcher before round 5) ran hipFuncSetAttribute in whichever
// lane thread launched the kernel first, concurrently with other lanes' launches and
// graph replays.
void set_lds_once(const void* kernel, int bytes) {
    static std::mutex mu;
    static std::set<const void*> done;
    std::lock_guard<std::mutex> lk(mu);
    if (done.insert(kernel).second) (void)hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// EPI_HEADS: the cross-K/V slot of window b of this GEMM (row refill encodes new windows
// into the slots of finished ones)
__device__ __forceinline__ int heads_window(const GemmArgs& g, int b) { return g.heads_slot ? g.heads_slot[b] : b; }

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// m / d for 0 <= m, 1 <= d.  Below 2^22 by a float reciprocal and one correction step
// (the estimate q·(1 ± 2^-22) is within 1 of the quotient there): ≈ 8 VALU instead of the
// ≈ 30 of an integer division (64-bit: more), which the tile epilogues did per output piece
// for the grouped-row and head-major addresses (90 division sequences in the fp32-residual
// kernel's ISA).  Exact either way.
__device__ __forceinline__ int fast_div(int m, int d) {
    if (m >= (1 << 22)) return m / d;
    int q = (int)((float)m * __builtin_amdgcn_rcpf((float)d));
    const int r = m - q * d;
    q += (r >= d ? 1 : 0) - (r < 0 ? 1 : 0);
    return q;
}

// element offset of output row m in the grouped layout (c_grp_rows rows per group,
// c_grp_stride elements between groups); one group: no division (a uniform branch)
__device__ __forceinline__ int64_t c_row(const GemmArgs& g, int m) {
    if (g.c_grp_rows >= g.M) return (int64_t)m * g.ldc;
    const int q = fast_div(m, g.c_grp_rows);
    return (int64_t)q * g.c_grp_stride + (int64_t)(m - q * g.c_grp_rows) * g.ldc;
}
// m's row within its group (the positional table's row for EPI_F32_GELU_POS)
__device__ __forceinline__ int c_rin(const GemmArgs& g, int m) {
    return g.c_grp_rows >= g.M ? m : m - fast_div(m, g.c_grp_rows) * g.c_grp_rows;
}

__device__ __forceinline__ const h16* grp_row(const h16* base, int64_t m, int64_t grp_rows, int64_t grp_stride,
                                              int64_t ld) {
    const int q = fast_div((int)m, (int)grp_rows);
    return base + (int64_t)q * grp_stride + (m - (int64_t)q * grp_rows) * ld;
}

template <int EPI>
__device__ __forceinline__ void store_one(const GemmArgs& g, int m, int n, float v) {
    if (g.bias) v += g.bias[n];
    const int64_t grp = fast_div(m, g.c_grp_rows), r = m - grp * g.c_grp_rows;
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
        const int which = fast_div(n, D), h = (n - which * D) >> 6, d = n & 63;
        const int bq = fast_div(m, g.heads_T);
                const int b = heads_window(g, bq), t = m - bq * g.heads_T;
        h16* C = (h16*)g.C;
        C[((((int64_t)which * g.heads_nb + b) * g.heads_H + h) * g.heads_T + t) * 64 + d] = (h16)v;
    }
}

// An accumulator's epilogue value, v + bias (hb: the GEMM has a bias), GELU'd for fc1
// (EPI_F32_GELU_POS: GELU + pos in the copy-out pass, fewer live registers).  The tile
// epilogues load the bias of a thread's columns into registers ONCE per tile: loading
// g.bias[n] per accumulator (rounds 1-5) re-loaded it behind every LDS image write (generic
// pointers: the compiler could not prove they do not alias, so it kept no value) and waited
// for each load with a full vmcnt(0) — 256-336 load/wait pairs per 8-phase tile epilogue in
// the ISA.  With no bias the register holds -0.0f, the exact additive identity of IEEE
// round-to-nearest (x + -0 == x for every x, -0 included), so the add is unconditional —
// a select on "has bias" was hoisted by the compiler across the passes and spilled.  Same
// arithmetic, bit for bit.
template <int EPI>
__device__ __forceinline__ float epi_apply(float v, float b) {
    v += b;
    if constexpr (EPI == EPI_F16_GELU) v = gelu_erf(v);
    return v;
}

// LDS-staged epilogue of a TM x TM tile held as 2 x 2 waves of (TM/2)^2 (gemm_kernel,
// gemm64_ring_kernel, gemm128_ring_kernel): bias / GELU applied into an LDS image of the
// tile (16-B chunks XOR-swizzled by row), then 16-B stores, TM*16 B per wave-instruction,
// instead of one 2-B / 4-B store per element (fc1's GELU tile at 4 windows: 172 us with
// per-element stores).  `smem` must hold TM*TM fp32 (every wave past its operand reads).
template <int EPI, int TM>
__device__ __forceinline__ void staged_epilogue_sq(const GemmArgs& g, const f32x4 (&acc)[TM / 32][TM / 32], int m0,
                                                   int n0, int wm, int wn, void* smem, int tid) {
    static_assert(EPI != EPI_F32, "plain fp32 tiles keep their write-through element stores");
    constexpr int FT = TM / 32, WT = TM / 2;
    const int lane = tid & 63;
    const bool hb = g.bias != nullptr;
    float bs[FT];  // the bias of this thread's FT columns, loaded once (epi_apply)
#pragma unroll
    for (int ni = 0; ni < FT; ++ni) bs[ni] = hb ? g.bias[min(n0 + wn * WT + ni * 16 + (lane & 15), g.N - 1)] : -0.f;
    if constexpr (EPI == EPI_F16 || EPI == EPI_F16_GELU || EPI == EPI_HEADS) {
        h16* T = (h16*)smem;
        auto at = [](int row, int col) { return row * TM + ((((col >> 3) ^ row) & (TM / 8 - 1)) << 3) + (col & 7); };
#pragma unroll
        for (int mi = 0; mi < FT; ++mi)
#pragma unroll
            for (int ni = 0; ni < FT; ++ni)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int row = wm * WT + mi * 16 + (lane >> 4) * 4 + i;
                    const int col = wn * WT + ni * 16 + (lane & 15);
                    T[at(row, col)] = (h16)epi_apply<EPI>(acc[mi][ni][i], bs[ni]);
                }
        __syncthreads();
#pragma unroll 4
        for (int j = 0; j < TM * TM / 8 / NTHR; ++j) {
            const int id = j * NTHR + tid;
            const int row = id / (TM / 8), c8 = (id % (TM / 8)) * 8;
            const int m = m0 + row, n = n0 + c8;
            if (m >= g.M || n >= g.N) continue;
            const h16x8 val = *(const h16x8*)&T[at(row, c8)];
            h16* dst;
            if constexpr (EPI == EPI_HEADS) {
                const int D = g.heads_H * 64;
                const int which = fast_div(n, D), h = (n - which * D) >> 6, d = n & 63;
                const int bq = fast_div(m, g.heads_T);
                const int b = heads_window(g, bq), t = m - bq * g.heads_T;
                dst = (h16*)g.C + ((((int64_t)which * g.heads_nb + b) * g.heads_H + h) * g.heads_T + t) * 64 + d;
            } else {
                dst = (h16*)g.C + c_row(g, m) + n;
            }
            *(h16x8*)dst = val;
        }
    } else {
        float* T = (float*)smem;
        auto at = [](int row, int col) { return row * TM + ((((col >> 2) ^ row) & (TM / 4 - 1)) << 2) + (col & 3); };
#pragma unroll
        for (int mi = 0; mi < FT; ++mi)
#pragma unroll
            for (int ni = 0; ni < FT; ++ni)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int row = wm * WT + mi * 16 + (lane >> 4) * 4 + i;
                    T[at(row, wn * WT + ni * 16 + (lane & 15))] = epi_apply<EPI>(acc[mi][ni][i], bs[ni]);
                }
        __syncthreads();
        // the residual (or positional) operands of every piece this thread stores are loaded
        // before any is used: one round trip, not one per piece
        constexpr int NJ = TM * TM / 4 / NTHR;
        f32x4 aux[EPI == EPI_F32_RESID || EPI == EPI_F32_GELU_POS ? NJ : 1];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int id = j * NTHR + tid;
            const int row = id / (TM / 4), c4 = (id % (TM / 4)) * 4;
            const int m = min(m0 + row, g.M - 1), n = min(n0 + c4, g.N - 4);
            if constexpr (EPI == EPI_F32_RESID)
                aux[j] = *(const f32x4*)((float*)g.C + c_row(g, m) + n);
            if constexpr (EPI == EPI_F32_GELU_POS) aux[j] = *(const f32x4*)&g.pos[(int64_t)c_rin(g, m) * g.N + n];
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int id = j * NTHR + tid;
            const int row = id / (TM / 4), c4 = (id % (TM / 4)) * 4;
            const int m = m0 + row, n = n0 + c4;
            if (m >= g.M || n >= g.N) continue;
            f32x4 val = *(const f32x4*)&T[at(row, c4)];
            float* dst = (float*)g.C + c_row(g, m) + n;
            if constexpr (EPI == EPI_F32_RESID) val += aux[j];
            if constexpr (EPI == EPI_F32_GELU_POS) {
#pragma unroll
                for (int e = 0; e < 4; ++e) val[e] = gelu_erf(val[e]) + aux[j][e];
            }
            *(f32x4*)dst = val;
        }
    }
}

// TM = 128 (the default) or 64: the 64x64 tile for small M (the encoder of one or a few
// windows: 1500 rows give a 128-tile N = 1280 GEMM only 120 workgroups for 256 CUs).
// Every output element is the same MFMA chain over K in the same order at either tile
// size (and in the 256-tile kernels), so the choice never changes a result.
template <int EPI, int TM = BM>
__global__ __launch_bounds__(NTHR, 2) void gemm_kernel(GemmArgs g) {
    constexpr int PW = TM / 32;  // glds pieces (8 rows x 128 B) per wave per operand
    constexpr int FT = TM / 32;  // 16x16 fragments per wave per dimension (2x2 waves)
    __shared__ __attribute__((aligned(16))) h16 lds[2][2][TM * BK];  // [buf][A|W]
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n0 = blockIdx.x * TM, m0 = blockIdx.y * TM;
    const int kc = g.kc > 0 ? g.kc : g.K, kbeg = blockIdx.z * kc;  // split-K: slab blockIdx.z

    // per-thread source rows for the A and W glds pieces (fixed over K)
    const h16* asrc[PW];
    const h16* wsrc[PW];
#pragma unroll
    for (int i = 0; i < PW; ++i) {
        const int r = (i * 4 + wave) * 8 + (lane >> 3);
        const int c = swz(r, lane & 7);
        const int gm = min(m0 + r, g.M - 1);
        const int gn = min(n0 + r, g.N - 1);
        asrc[i] = grp_row(g.A, gm, g.a_grp_rows, g.a_grp_stride, g.lda) + c * 8 + kbeg;
        wsrc[i] = g.W + (int64_t)gn * g.ldw + c * 8 + kbeg;
    }

    auto stage = [&](int buf, int k0) {
#pragma unroll
        for (int i = 0; i < PW; ++i) {
            h16* da = &lds[buf][0][(i * 4 + wave) * 8 * BK];
            h16* dw = &lds[buf][1][(i * 4 + wave) * 8 * BK];
            __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + k0), (OSW_LDS void*)da, 16, 0, 0);
            __builtin_amdgcn_global_load_lds((const void*)(wsrc[i] + k0), (OSW_LDS void*)dw, 16, 0, 0);
        }
    };

    const int wm = wave >> 1, wn = wave & 1;
    constexpr int WT = TM / 2;  // wave tile edge
    f32x4 acc[FT][FT];
#pragma unroll
    for (int i = 0; i < FT; ++i)
#pragma unroll
        for (int j = 0; j < FT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = kc / BK;
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
            h16x8 a[FT], b[FT];
#pragma unroll
            for (int mi = 0; mi < FT; ++mi) {
                const int row = wm * WT + mi * 16 + (lane & 15);
                a[mi] = *(const h16x8*)&la[row * BK + swz(row, c) * 8];
            }
#pragma unroll
            for (int ni = 0; ni < FT; ++ni) {
                const int row = wn * WT + ni * 16 + (lane & 15);
                b[ni] = *(const h16x8*)&lw[row * BK + swz(row, c) * 8];
            }
#pragma unroll
            for (int mi = 0; mi < FT; ++mi)
#pragma unroll
                for (int ni = 0; ni < FT; ++ni)
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
        }
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
    }

    if (EPI == EPI_F32 && g.kc > 0) {  // split-K partial slab: plain stores, no bias
        float* C = (float*)g.C + (int64_t)blockIdx.z * g.M * g.ldc;
#pragma unroll
        for (int mi = 0; mi < FT; ++mi)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int m = m0 + wm * WT + mi * 16 + (lane >> 4) * 4 + i;
                if (m >= g.M) continue;
#pragma unroll
                for (int ni = 0; ni < FT; ++ni) {
                    const int n = n0 + wn * WT + ni * 16 + (lane & 15);
                    if (n < g.N)  // written through L2, like the skinny slabs
                        __hip_atomic_store(&C[(int64_t)m * g.ldc + n], acc[mi][ni][i], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        return;
    }
    if constexpr (EPI != EPI_F32) {  // 16-B chunk stores through an LDS image (loop drained: LDS free)
        staged_epilogue_sq<EPI, TM>(g, acc, m0, n0, wm, wn, &lds[0][0][0], threadIdx.x);
        return;
    }
#pragma unroll
    for (int mi = 0; mi < FT; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = m0 + wm * WT + mi * 16 + (lane >> 4) * 4 + i;
            if (m >= g.M) continue;
#pragma unroll
            for (int ni = 0; ni < FT; ++ni) {
                const int n = n0 + wn * WT + ni * 16 + (lane & 15);
                if (n >= g.N) continue;
                if constexpr (EPI == EPI_F32) {  // decoder logits: written through L2 for the select kernels
                    const float v = g.bias ? acc[mi][ni][i] + g.bias[n] : acc[mi][ni][i];
                    const int64_t grp = fast_div(m, g.c_grp_rows), r = m - grp * g.c_grp_rows;
                    __hip_atomic_store((float*)g.C + grp * g.c_grp_stride + r * g.ldc + n, v, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                } else
                    store_one<EPI>(g, m, n, acc[mi][ni][i]);
            }
        }
}
// ---------------------------------------------------------------------------
// Large-M variant (encoder at batch >= ~8 windows): 256x256x64 tile, 8 waves (2 x 4),
// each wave 128x64 = 8x4 MFMA tiles.  One K-step is 2048 MFMA cycles per SIMD
// (~0.85 us), long enough to hide the one-tile-ahead global_load_lds prefetch that
// the 128x128 tile (~0.2 us per K-step) cannot.  128 KiB LDS (2 stages) -> one
// workgroup per CU.  Tiles are walked XCD-aware: the dispatcher deals workgroups
// round-robin over the 8 XCDs, so id b is remapped to tile (b % 8)*ceil(n/8) + b/8
// (bijective form) and each XCD's L2 sees a contiguous run of tiles that share
// A row-panels.
constexpr int GB = 256, GNT = 512;

// LDS-staged epilogue for the 256x256 tile: the accumulators (bias / GELU / pos
// applied) are written to an LDS image of the tile, then every thread streams 16-B
// chunks to global — 1 KiB contiguous per wave-instruction instead of 128 scattered
// 2/4-B stores per lane.  fp32 tiles go through LDS in two 128-row halves.  The image
// rows are unpadded with the 16-B chunk XOR-swizzled by row (conflict-free MFMA-layout
// writes: the 4 rows of one write are 4 apart, so their chunks land on distinct banks),
// so the image is exactly the 128 KiB operand ring: the kernel leaves 32 KiB of the
// CU's LDS free, enough for a co-resident decoder workgroup of another lane (a padded
// 135 KiB image left 28 KiB, which no skinny GEMM workgroup fits: the decoder's
// projections then waited for whole encoder tiles to retire).
constexpr int EPI_LDS = 256 * 256 * 2;  // 131072 B = 128 rows x 256 fp32
__device__ __forceinline__ int ep16(int row, int col) { return row * 256 + ((((col >> 3) ^ row) & 31) << 3) + (col & 7); }
__device__ __forceinline__ int ep32(int row, int col) { return row * 256 + ((((col >> 2) ^ row) & 63) << 2) + (col & 3); }


// IL = false: wave (wm, wn) owns rows wm*128 + [0,128) and cols wn*64 + [0,64).
// IL = true (8-phase kernel): rows {0,128} + wm*64 + [0,64), cols {0,128} + wn*32 + [0,32).
template <bool IL>
__device__ __forceinline__ int acc_row(int wm, int mi) { return IL ? (mi >> 2) * 128 + wm * 64 + (mi & 3) * 16 : wm * 128 + mi * 16; }
template <bool IL>
__device__ __forceinline__ int acc_col(int wn, int ni) { return IL ? (ni >> 1) * 128 + wn * 32 + (ni & 1) * 16 : wn * 64 + ni * 16; }

// Output rows leave through nontemporal stores: the encoder's activations (0.5-2 GB per
// GEMM at 64 windows) stream past the MALL instead of evicting the weights and the
// next GEMM's operand panels (8p GEMMs 4-7 % and the attention after them 6 % faster).
// TR (8-phase kernel, IL, fp16 epilogues): the accumulators are transposed (the kernel swaps
// the MFMA operands), lane l of block (mi, ni) holding C[row + (l & 15)][col + 4 (l >> 4) + e],
// so the image takes one 8-B write per block instead of four 2-B ones
// (fc1 at 64 windows 1488 -> 1432 us, + GELU 1694 -> 1627 us; profiles/r04_s_epilogue.jsonl, r04_t_epilogue_forms.jsonl)
// TN: the tile's width (256; 128 for the half-width tile, whose waves hold accumulator
// blocks ni < 2 only): the image keeps its 256-wide rows, the copy-out covers TN columns
template <int EPI, bool IL = false, bool TR = false, int TN = 256>
__device__ __forceinline__ void staged_epilogue(const GemmArgs& g, f32x4 (&acc)[8][4], int m0, int n0, int wm,
                                                int wn, char* smem, int tid) {
    static_assert(TN == 256 || (TN == 128 && IL), "the half-width tile is the 8-phase layout");
    constexpr int NI = TN / 64;        // accumulator column blocks per wave
    constexpr int C16 = TN / 8;        // 16-B fp16 chunks per image row
    constexpr int C32 = TN / 4;        // 16-B fp32 chunks per image row
    // (shifts and masks, not / and %: on the signed thread index those cost a sign fix-up each,
    // which pushed the fp32-residual 8-phase epilogue from 250 VGPRs to 256 + 49 spilled)
    constexpr int L16 = TN == 256 ? 5 : 4, L32 = TN == 256 ? 6 : 5;
    const int lane = tid & 63;
    // the bias of this thread's columns, loaded once per tile (epi_apply): TR, 4 columns per
    // accumulator block (one 16-B load each); otherwise one column per block
    // (fp32 forms: one f32x4 per thread, added at copy-out, whose columns are fixed per thread)
    constexpr bool F16 = EPI == EPI_F16 || EPI == EPI_F16_GELU || EPI == EPI_HEADS;
    const bool hb = g.bias != nullptr;
    f32x4 bt[4];
    float bs[4];
#pragma unroll
    for (int ni = 0; ni < NI && F16; ++ni) {
        if constexpr (TR) {
            const int n = min(n0 + acc_col<IL>(wn, ni) + 4 * (lane >> 4), g.N - 4);
            bt[ni] = hb ? *(const f32x4*)(g.bias + n) : f32x4{-0.f, -0.f, -0.f, -0.f};
        } else {
            bs[ni] = hb ? g.bias[min(n0 + acc_col<IL>(wn, ni) + (lane & 15), g.N - 1)] : -0.f;
        }
    }
    __syncthreads();
    if constexpr (EPI == EPI_F16 || EPI == EPI_F16_GELU || EPI == EPI_HEADS) {
        // IL (every wave holds rows of both 128-row halves): the tile leaves in two halves,
        // so the second half's bias/GELU (VALU) runs while the first half's stores drain
        // (the whole grid reaches its epilogue together: the stores are HBM-bound there)
        h16* T = (h16*)smem;
        constexpr int NH = IL ? 2 : 1;
#pragma unroll
        for (int half = 0; half < NH; ++half) {
        if constexpr (TR) {
#pragma unroll
            for (int mi = 0; mi < 8; ++mi)
#pragma unroll
                for (int ni = 0; ni < NI; ++ni) {
                    if (IL && (mi >> 2) != half) continue;
                    const int row = acc_row<IL>(wm, mi) + (lane & 15);
                    const int col = acc_col<IL>(wn, ni) + 4 * (lane >> 4);
                    h16x4 v;
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = (h16)epi_apply<EPI>(acc[mi][ni][e], bt[ni][e]);
                    *(h16x4*)&T[ep16(row, col)] = v;
                }
        } else
#pragma unroll
        for (int mi = 0; mi < 8; ++mi)
#pragma unroll
            for (int ni = 0; ni < NI; ++ni)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    if (IL && (mi >> 2) != half) continue;
                    const int row = acc_row<IL>(wm, mi) + (lane >> 4) * 4 + i;
                    const int col = acc_col<IL>(wn, ni) + (lane & 15);
                    T[ep16(row, col)] = (h16)epi_apply<EPI>(acc[mi][ni][i], bs[ni]);
                }
        __syncthreads();
#pragma unroll 4
        for (int j = 0; j < 256 * C16 / GNT / NH; ++j) {
            const int id = j * GNT + tid;
            const int row = half * 128 + (id >> L16), c8 = (id & (C16 - 1)) * 8;
            const int m = m0 + row, n = n0 + c8;
            if (m >= g.M || n >= g.N) continue;
            const h16x8 v = *(const h16x8*)&T[ep16(row, c8)];
            h16* dst;
            if constexpr (EPI == EPI_HEADS) {
                const int D = g.heads_H * 64;
                const int which = fast_div(n, D), h = (n - which * D) >> 6, d = n & 63;
                const int bq = fast_div(m, g.heads_T);
                const int b = heads_window(g, bq), t = m - bq * g.heads_T;
                dst = (h16*)g.C + ((((int64_t)which * g.heads_nb + b) * g.heads_H + h) * g.heads_T + t) * 64 + d;
            } else {
                dst = (h16*)g.C + c_row(g, m) + n;
            }
            __builtin_nontemporal_store(v, (h16x8*)dst);
        }
        }
    } else {
        float* T = (float*)smem;
        // this thread's 4 copy-out columns are the same in every piece (GNT % 64 == 0)
        const f32x4 b4 = hb ? *(const f32x4*)(g.bias + min(n0 + (tid & (C32 - 1)) * 4, g.N - 4))
                            : f32x4{-0.f, -0.f, -0.f, -0.f};
        for (int half = 0; half < 2; ++half) {
            if (IL || wm == half) {
#pragma unroll
                for (int mi = 0; mi < 8; ++mi)
#pragma unroll
                    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            if (IL && (mi >> 2) != half) continue;
                            const int row = acc_row<IL>(wm, mi) - half * 128 + (lane >> 4) * 4 + i;
                            const int col = acc_col<IL>(wn, ni) + (lane & 15);
                            T[ep32(row, col)] = acc[mi][ni][i];
                        }
            }
            __syncthreads();
            // the residual (positional) operands of AB pieces in flight at once: 16 / AB round
            // trips per half instead of one per piece (each piece's load was followed by a full
            // vmcnt(0) wait, which also waited for the previous piece's store).  AB = 8 when
            // only the other half's accumulators are live (IL); 1 when all are (more spilled).
            constexpr int AB = IL ? 8 : 1;
            constexpr int NJ = 128 * C32 / GNT;  // pieces per thread per half
#pragma unroll
            for (int j0 = 0; j0 < NJ; j0 += AB) {
            f32x4 aux[EPI == EPI_F32_RESID || EPI == EPI_F32_GELU_POS ? AB : 1];
#pragma unroll
            for (int jj = 0; jj < AB; ++jj) {
                const int id = (j0 + jj) * GNT + tid;
                const int row = id >> L32, c4 = (id & (C32 - 1)) * 4;
                const int m = min(m0 + half * 128 + row, g.M - 1), n = min(n0 + c4, g.N - 4);
                if constexpr (EPI == EPI_F32_RESID)
                    aux[jj] = *(const f32x4*)((float*)g.C + c_row(g, m) + n);
                if constexpr (EPI == EPI_F32_GELU_POS)
                    aux[jj] = *(const f32x4*)&g.pos[(int64_t)c_rin(g, m) * g.N + n];
            }
#pragma unroll
            for (int jj = 0; jj < AB; ++jj) {
                const int j = j0 + jj;
                const int id = j * GNT + tid;
                const int row = id >> L32, c4 = (id & (C32 - 1)) * 4;
                const int m = m0 + half * 128 + row, n = n0 + c4;
                if (m < g.M && n < g.N) {
                    f32x4 v = *(const f32x4*)&T[ep32(row, c4)] + b4;
                    float* dst = (float*)g.C + c_row(g, m) + n;
                    if constexpr (EPI == EPI_F32_RESID) v += aux[jj];
                    if constexpr (EPI == EPI_F32_GELU_POS) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = gelu_erf(v[e]) + aux[jj][e];
                    }
                    __builtin_nontemporal_store(v, (f32x4*)dst);
                }
            }
            }
            __syncthreads();
        }
    }
}

template <int EPI>
__global__ __launch_bounds__(GNT, 1) void gemm256_kernel(GemmArgs g) {
    extern __shared__ __attribute__((aligned(16))) h16 smem[];  // [2][A|W][256*64]
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int ntn = (g.N + GB - 1) / GB, ntm = (g.M + GB - 1) / GB;
    const int nwg = ntn * ntm;
    const int bid = blockIdx.x;
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
    const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    // column bands of G tiles: consecutive tiles sweep G columns of one row panel, then
    // the next row panel, so an XCD keeps G weight panels L2-hot while A panels stream
    // (G chosen on the host to minimise A*ntn/G + W*ntm*G/32 bytes of L2 misses)
    const int G = g.band > 0 ? min(g.band, ntn) : ntn;
    const int band = tile / (G * ntm), rr0 = tile % (G * ntm);
    const int gw = min(G, ntn - band * G);
    const int n0 = (band * G + rr0 % gw) * GB, m0 = (rr0 / gw) * GB;

    const h16* asrc[4];
    const h16* wsrc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int rr = (i * 8 + wave) * 8 + (lane >> 3);
        const int c = swz(rr, lane & 7);
        asrc[i] = grp_row(g.A, min(m0 + rr, g.M - 1), g.a_grp_rows, g.a_grp_stride, g.lda) + c * 8;
        wsrc[i] = g.W + (int64_t)min(n0 + rr, g.N - 1) * g.ldw + c * 8;
    }
    auto stage = [&](int buf, int k0) {
        h16* base = smem + buf * (2 * GB * BK);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int piece = i * 8 + wave;
            __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + k0), (OSW_LDS void*)(base + piece * 8 * BK),
                                             16, 0, 0);
            __builtin_amdgcn_global_load_lds((const void*)(wsrc[i] + k0),
                                             (OSW_LDS void*)(base + GB * BK + piece * 8 * BK), 16, 0, 0);
        }
    };
    const int wm = wave >> 2, wn = wave & 3;
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = g.K / BK;
    stage(0, 0);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) stage(buf ^ 1, (kt + 1) * BK);
        const h16* la = smem + buf * (2 * GB * BK);
        const h16* lw = la + GB * BK;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int c = ks * 4 + (lane >> 4);
            h16x8 b[4];
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) {
                const int row = wn * 64 + ni * 16 + (lane & 15);
                b[ni] = *(const h16x8*)&lw[row * BK + swz(row, c) * 8];
            }
#pragma unroll
            for (int mi = 0; mi < 8; ++mi) {
                const int row = wm * 128 + mi * 16 + (lane & 15);
                const h16x8 a = *(const h16x8*)&la[row * BK + swz(row, c) * 8];
#pragma unroll
                for (int ni = 0; ni < 4; ++ni)
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b[ni], acc[mi][ni], 0, 0, 0);
            }
        }
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
    }
    staged_epilogue<EPI>(g, acc, m0, n0, wm, wn, (char*)smem, threadIdx.x);
}

// band width minimising modelled L2-miss bytes: A re-read once per band, a band's
// weights re-read once per 32/G concurrently resident row panels of an XCD
int choose_band(const GemmArgs& g, int tn = GB) {
    if (const char* e = getenv("OSW_GEMM_BAND")) return atoi(e);
    const int ntn = (g.N + tn - 1) / tn, ntm = (g.M + GB - 1) / GB;
    const double abytes = (double)g.M * g.K * 2, wbytes = (double)g.N * g.K * 2;
    int best = ntn;
    double bc = 1e300;
    for (int G = 1; G <= ntn; ++G) {
        const double c = abytes * ((ntn + G - 1) / G) + wbytes * ntm * G / 32.0;
        if (c < bc) { bc = c; best = G; }
    }
    return best;
}

template <int EPI>
void launch256(const GemmArgs& g0, hipStream_t s) {
    constexpr int lds = EPI_LDS > 2 * 2 * GB * BK * 2 ? EPI_LDS : 2 * 2 * GB * BK * 2;
    set_lds_once((const void*)gemm256_kernel<EPI>, lds);
    GemmArgs g = g0;
    g.band = choose_band(g);
    const int nwg = ((g.N + GB - 1) / GB) * ((g.M + GB - 1) / GB);
    gemm256_kernel<EPI><<<nwg, GNT, lds, s>>>(g);
}

// 8-phase ping-pong variant (cdna_hip_programming.md §5 "The 256² 8-phase template",
// T3-T5).  Same 256x256x64 tile and 8 waves, but the K-tile is split into four
// phases of 16 MFMAs (one 64x32 quadrant of the wave's output each), separated by
// raw s_barriers, and the two 4-wave groups (wm = 0 / 1) run one barrier apart: in
// every barrier interval one group is in its MFMA cluster while the other issues
// its ds_reads and global_load_lds, so each SIMD's matrix pipe alternates between
// its two waves instead of idling through a shared load/wait step.
//
// Wave (wm, wn) owns rows {0,128} + wm*64 + [0,64) and cols {0,128} + wn*32 + [0,32),
// so quadrant (a, b) reads only half-tile A_a (A rows a*128..) and W_b.  LDS holds
// 2 buffers x 4 half-tiles {A0, A1, W0, W1} x 16 KiB.  Per K-tile t the phases
// read:  1: A0 + W0   2: W1   3: A1   4: W0 (A1 kept in registers).
// Every half-tile slot is restaged as soon as it is 2 phases past its last read:
//   phase 1 stages A1(t+1), 2: W0(t+1), 3: A0(t+2), 4: W1(t+2)
// and phase 4 waits vmcnt(4) (A0(t+2), W1(t+2) stay in flight), which retires all
// of tile t+1 one phase before its first read.  The global_load_lds stream is never
// drained inside the loop (raw s_barrier, no __syncthreads).
constexpr int HT = 128 * BK;  // halfs per half-tile

// tile origin of virtual workgroup id `bid` (XCD-contiguous runs, column bands of G tiles)
// (TN: the tile's width, 256 or 128 for the half-width tile gemm8h_kernel)
template <int TN = GB>
__device__ __forceinline__ void tile8p_origin(const GemmArgs& g, int bid, int& m0, int& n0) {
    const int ntn = (g.N + TN - 1) / TN, ntm = (g.M + GB - 1) / GB;
    const int nwg = ntn * ntm;
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
    const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
    const int G = g.band > 0 ? min(g.band, ntn) : ntn;
    const int band = tile / (G * ntm), rr0 = tile % (G * ntm);
    const int gw = min(G, ntn - band * G);
    n0 = (band * G + rr0 % gw) * TN;
    m0 = (rr0 / gw) * GB;
}

// glds source of half-tile H (0, 1: A rows m0 + 128 H; 2, 3: W rows n0 + 128 (H - 2)),
// piece i*8 + wave (8 rows of 128 B), lane -> row, swizzled chunk
__device__ __forceinline__ const h16* src8p(const GemmArgs& g, int m0, int n0, int H, int i, int wave, int lane) {
    const int rr = (i * 8 + wave) * 8 + (lane >> 3);
    const int c = swz(rr, lane & 7);
    const int hh = H & 1;
    if (H < 2) return grp_row(g.A, min(m0 + hh * 128 + rr, g.M - 1), g.a_grp_rows, g.a_grp_stride, g.lda) + c * 8;
    return g.W + (int64_t)min(n0 + hh * 128 + rr, g.N - 1) * g.ldw + c * 8;
}

__device__ __forceinline__ void lds_sync() {  // LDS accesses of every wave done, vmcnt untouched
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// The persistent 8-phase kernel's epilogue when the next tile's first K-tile is already
// in flight into ring buffer 0 (NEXT0): the image lives in buffer 1 (the upper 64 KiB) and
// the tile leaves in passes that fit it — fp16: two 128-row halves, fp32: four 64-row
// quarters — with LDS-only barriers, so the prefetch loads stay in flight throughout.
template <int EPI, bool TR = false>
__device__ __forceinline__ void staged_epilogue_next0(const GemmArgs& g, f32x4 (&acc)[8][4], int m0, int n0, int wm,
                                                      int wn, char* smem, int tid) {
    const int lane = tid & 63;
    constexpr bool F16 = EPI == EPI_F16 || EPI == EPI_F16_GELU || EPI == EPI_HEADS;
    constexpr int PR = F16 ? 128 : 64;       // image rows per pass
    constexpr int NP = 256 / PR;
    // the bias of this thread's columns, loaded once per tile (epi_apply; see staged_epilogue)
    const bool hb = g.bias != nullptr;
    f32x4 bt[4];
    float bs[4];
#pragma unroll
    for (int ni = 0; ni < 4 && F16; ++ni) {
        if constexpr (TR) {
            const int n = min(n0 + acc_col<true>(wn, ni) + 4 * (lane >> 4), g.N - 4);
            bt[ni] = hb ? *(const f32x4*)(g.bias + n) : f32x4{-0.f, -0.f, -0.f, -0.f};
        } else {
            bs[ni] = hb ? g.bias[min(n0 + acc_col<true>(wn, ni) + (lane & 15), g.N - 1)] : -0.f;
        }
    }
    lds_sync();  // every wave is past its last read of buffer 1 (the last K-tile's)
#pragma unroll
    for (int pass = 0; pass < NP; ++pass) {
        if constexpr (F16) {
            h16* T = (h16*)(smem + 4 * HT * 2);
            if constexpr (TR) {
#pragma unroll
                for (int mi = 0; mi < 8; ++mi)
#pragma unroll
                    for (int ni = 0; ni < 4; ++ni) {
                        if ((mi >> 2) != pass) continue;
                        const int row = acc_row<true>(wm, mi) - pass * PR + (lane & 15);
                        const int col = acc_col<true>(wn, ni) + 4 * (lane >> 4);
                        h16x4 v;
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = (h16)epi_apply<EPI>(acc[mi][ni][e], bt[ni][e]);
                        *(h16x4*)&T[ep16(row, col)] = v;
                    }
            } else
#pragma unroll
            for (int mi = 0; mi < 8; ++mi)
#pragma unroll
                for (int ni = 0; ni < 4; ++ni)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        if ((mi >> 2) != pass) continue;
                        const int row = acc_row<true>(wm, mi) - pass * PR + (lane >> 4) * 4 + i;
                        const int col = acc_col<true>(wn, ni) + (lane & 15);
                        T[ep16(row, col)] = (h16)epi_apply<EPI>(acc[mi][ni][i], bs[ni]);
                    }
            lds_sync();
#pragma unroll 4
            for (int j = 0; j < 8; ++j) {
                const int id = j * GNT + tid;
                const int row = id >> 5, c8 = (id & 31) * 8;
                const int m = m0 + pass * PR + row, n = n0 + c8;
                if (m >= g.M || n >= g.N) continue;
                const h16x8 v = *(const h16x8*)&T[ep16(row, c8)];
                h16* dst;
                if constexpr (EPI == EPI_HEADS) {
                    const int D = g.heads_H * 64;
                    const int which = fast_div(n, D), h = (n - which * D) >> 6, d = n & 63;
                    const int bq = fast_div(m, g.heads_T);
                const int b = heads_window(g, bq), t = m - bq * g.heads_T;
                    dst = (h16*)g.C + ((((int64_t)which * g.heads_nb + b) * g.heads_H + h) * g.heads_T + t) * 64 + d;
                } else {
                    dst = (h16*)g.C + c_row(g, m) + n;
                }
                __builtin_nontemporal_store(v, (h16x8*)dst);
            }
        } else {
            float* T = (float*)(smem + 4 * HT * 2);
            const f32x4 b4 = hb ? *(const f32x4*)(g.bias + min(n0 + (tid & 63) * 4, g.N - 4))
                                : f32x4{-0.f, -0.f, -0.f, -0.f};
            // pass p = rows [64 p, 64 p + 64): wave rows (mi >> 2) * 128 + wm * 64
            if (wm == (pass & 1)) {
#pragma unroll
                for (int mi = 0; mi < 8; ++mi)
#pragma unroll
                    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            if ((mi >> 2) != (pass >> 1)) continue;
                            const int row = acc_row<true>(wm, mi) - pass * PR + (lane >> 4) * 4 + i;
                            const int col = acc_col<true>(wn, ni) + (lane & 15);
                            T[ep32(row, col)] = acc[mi][ni][i];
                        }
            }
            lds_sync();
            // the residual (positional) operands in flight 4 at a time: every accumulator is
            // still live here (later passes), so 8 at a time spilled
#pragma unroll
            for (int j0 = 0; j0 < 8; j0 += 4) {
                f32x4 aux[EPI == EPI_F32_RESID || EPI == EPI_F32_GELU_POS ? 4 : 1];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const int id = (j0 + jj) * GNT + tid;
                    const int row = id >> 6, c4 = (id & 63) * 4;
                    const int m = min(m0 + pass * PR + row, g.M - 1), n = min(n0 + c4, g.N - 4);
                    if constexpr (EPI == EPI_F32_RESID)
                        aux[jj] = *(const f32x4*)((float*)g.C + c_row(g, m) + n);
                    if constexpr (EPI == EPI_F32_GELU_POS)
                        aux[jj] = *(const f32x4*)&g.pos[(int64_t)c_rin(g, m) * g.N + n];
                }
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const int id = (j0 + jj) * GNT + tid;
                    const int row = id >> 6, c4 = (id & 63) * 4;
                    const int m = m0 + pass * PR + row, n = n0 + c4;
                    if (m < g.M && n < g.N) {
                        f32x4 v = *(const f32x4*)&T[ep32(row, c4)] + b4;
                        float* dst = (float*)g.C + c_row(g, m) + n;
                        if constexpr (EPI == EPI_F32_RESID) v += aux[jj];
                        if constexpr (EPI == EPI_F32_GELU_POS) {
#pragma unroll
                            for (int e = 0; e < 4; ++e) v[e] = gelu_erf(v[e]) + aux[jj][e];
                        }
                        __builtin_nontemporal_store(v, (f32x4*)dst);
                    }
                }
            }
        }
        lds_sync();  // the image's reads are done before the next pass (or the next tile) writes it
    }
}

// NEXT0: K-tile 0 of this tile was staged by the previous tile (pre0) / stage the next
// tile's K-tile 0 (next_bid >= 0) before this tile's epilogue
template <int EPI, int DBG>
__device__ __forceinline__ void gemm8p_tile(const GemmArgs& g, int bid, h16* smem, int tid, bool pre0 = false,
                                            int next_bid = -1) {
    const int wave = tid >> 6, lane = tid & 63;
    // transposed accumulators for the fp16 epilogues only: the fp32 and head-major forms
    // need 217-219 VGPRs transposed (213-216 plain), which rounds the allocation up to 224
    // and leaves 64 instead of 80 VGPRs per SIMD, too few for a 74-VGPR decoder
    // cross-attention wave of another lane to sit beside the encoder workgroup (§5.3.1)
    constexpr bool TR = DBG != 2 && (EPI == EPI_F16 || EPI == EPI_F16_GELU);
    int m0, n0;
    tile8p_origin(g, bid, m0, n0);

    const h16* src[4][2];
#pragma unroll
    for (int H = 0; H < 4; ++H)
#pragma unroll
        for (int i = 0; i < 2; ++i) src[H][i] = src8p(g, m0, n0, H, i, wave, lane);
    auto stage = [&](int H, int t) {
        h16* base = smem + ((t & 1) * 4 + H) * HT;
#pragma unroll
        for (int i = 0; i < 2; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(src[H][i] + t * BK),
                                             (OSW_LDS void*)(base + (i * 8 + wave) * 8 * BK), 16, 0, 0);
    };
    const int wm = wave >> 2, wn = wave & 3;
    const int li = lane & 15, lc = lane >> 4;
    // per-lane LDS element offsets of the fragment reads (swizzle is the same for every 16-row step)
    const int aoff0 = (wm * 64 + li) * BK + swz(wm * 64 + li, lc) * 8;
    const int aoff1 = (wm * 64 + li) * BK + swz(wm * 64 + li, 4 + lc) * 8;
    const int boff0 = (wn * 32 + li) * BK + swz(wn * 32 + li, lc) * 8;
    const int boff1 = (wn * 32 + li) * BK + swz(wn * 32 + li, 4 + lc) * 8;

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // KW (DBG 3, 4): W0's fragments stay in registers (bw) from phase 1 to phase 4
    constexpr bool KW = DBG == 3 || DBG == 4;
    constexpr bool NOEPI = DBG == 1 || DBG == 4;
    h16x8 af[4][2], bf[2][2], bw[KW ? 2 : 1][2];

    auto read_a = [&](const h16* hb) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
            af[mt][0] = *(const h16x8*)&hb[aoff0 + mt * 16 * BK];
            af[mt][1] = *(const h16x8*)&hb[aoff1 + mt * 16 * BK];
        }
    };
    auto read_b = [&](const h16* hb) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
            bf[nt][0] = *(const h16x8*)&hb[boff0 + nt * 16 * BK];
            bf[nt][1] = *(const h16x8*)&hb[boff1 + nt * 16 * BK];
        }
    };
    auto read_w0 = [&](const h16* hb) {
#pragma unroll
        for (int nt = 0; nt < (KW ? 2 : 0); ++nt) {
            bw[nt][0] = *(const h16x8*)&hb[boff0 + nt * 16 * BK];
            bw[nt][1] = *(const h16x8*)&hb[boff1 + nt * 16 * BK];
        }
    };
    auto barrier = [] {
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    auto mfma_with = [&](int a, int b, const h16x8 (&B)[2][2]) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {
                f32x4 c = acc[a * 4 + mt][b * 2 + nt];
                if constexpr (TR) {  // transposed: Cᵀ = W Aᵀ, the same products in the same K order
                    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(B[nt][0], af[mt][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(B[nt][1], af[mt][1], c, 0, 0, 0);
                } else {
                    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[mt][0], B[nt][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[mt][1], B[nt][1], c, 0, 0, 0);
                }
                acc[a * 4 + mt][b * 2 + nt] = c;
            }
        __builtin_amdgcn_s_setprio(0);
    };
    auto mfma = [&](int a, int b) { mfma_with(a, b, bf); };

    const int nk = g.K / BK;
    if constexpr (KW) {
        // Issue order per K-tile t: phase 1 W1(t+1), 2 A1(t+1), 3 A0(t+2), 4 W0(t+2); every
        // half-tile slot is restaged 2-3 phases after its last read (W0's last read is phase 1)
        // and waited for 4 phases after its issue (vmcnt(8): the 4 younger half-tiles stay in
        // flight), in the phase before the one that reads it:
        //   phase 1 retires W1(t) (read in 2), 2 A1(t) (read in 3), 4 A0(t+1) + W0(t+1).
        // (The default order re-reads W0 in phase 4, which holds W0(t+1)'s restage back to
        // phase 2 and leaves it 2 phases to arrive.)
        if (!pre0) {
            stage(0, 0);
            stage(2, 0);
            stage(3, 0);
            stage(1, 0);
        }
        if (nk > 1) {
            stage(0, 1);
            stage(2, 1);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        }
        barrier();
        if (__builtin_amdgcn_readfirstlane(wave) >= 4) barrier();  // group 1 runs one barrier behind group 0
        for (int t = 0; t < nk; ++t) {
            const h16* buf = smem + (t & 1) * 4 * HT;
            const bool n1 = t + 1 < nk, n2 = t + 2 < nk;
            // phase 1: quadrant (0,0) from A0, W0 (W0 kept)
            if (n1) stage(3, t + 1);
            read_a(buf + 0 * HT);
            read_w0(buf + 2 * HT);
            if (n1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
            barrier();
            mfma_with(0, 0, bw);
            barrier();
            // phase 2: quadrant (0,1) from W1
            if (n1) stage(1, t + 1);
            read_b(buf + 3 * HT);
            if (n1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            barrier();
            mfma(0, 1);
            barrier();
            // phase 3: quadrant (1,1) from A1
            if (n2) stage(0, t + 2);
            read_a(buf + 1 * HT);
            barrier();
            mfma(1, 1);
            barrier();
            // phase 4: quadrant (1,0), no reads
            if (n2) {
                stage(2, t + 2);
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            } else if (n1) {
                asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            barrier();
            mfma_with(1, 0, bw);
            barrier();
        }
    } else {
    // prologue = phases 3, 4 of tile -2 and tile -1 in the steady-state order
    if (!pre0) {
        stage(0, 0);
        stage(3, 0);
        stage(1, 0);
        stage(2, 0);
    }
    if (nk > 1) {
        stage(0, 1);
        stage(3, 1);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    barrier();
    if (__builtin_amdgcn_readfirstlane(wave) >= 4) barrier();  // group 1 runs one barrier behind group 0

    for (int t = 0; t < nk; ++t) {
        const h16* buf = smem + (t & 1) * 4 * HT;
        const bool n1 = t + 1 < nk, n2 = t + 2 < nk;
        // phase 1: quadrant (0,0)
        if (n1) stage(1, t + 1);
        read_a(buf + 0 * HT);
        read_b(buf + 2 * HT);
        barrier();
        mfma(0, 0);
        barrier();
        // phase 2: quadrant (0,1)
        if (n1) stage(2, t + 1);
        read_b(buf + 3 * HT);
        barrier();
        mfma(0, 1);
        barrier();
        // phase 3: quadrant (1,1)
        if (n2) stage(0, t + 2);
        read_a(buf + 1 * HT);
        barrier();
        mfma(1, 1);
        barrier();
        // phase 4: quadrant (1,0); retire tile t+1
        if (n2) {
            stage(3, t + 2);
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        read_b(buf + 2 * HT);
        barrier();
        mfma(1, 0);
        barrier();
    }
    }
    if (__builtin_amdgcn_readfirstlane(wave) < 4) barrier();
    if (next_bid >= 0) {
        // every wave is past its reads of buffer 0 (the last K-tile read buffer 1: nk even):
        // the next tile's K-tile 0 streams in while this tile's epilogue runs in buffer 1
        lds_sync();
        int nm0, nn0;
        tile8p_origin(g, next_bid, nm0, nn0);
        // (the prologue's issue order: A0 W1 A1 W0, KW: A0 W0 W1 A1)
        constexpr int H0 = 0, H1 = KW ? 2 : 3, H2 = KW ? 3 : 1, H3 = KW ? 1 : 2;
#pragma unroll
        for (int H : {H0, H1, H2, H3})
#pragma unroll
            for (int i = 0; i < 2; ++i)
                __builtin_amdgcn_global_load_lds((const void*)src8p(g, nm0, nn0, H, i, wave, lane),
                                                 (OSW_LDS void*)(smem + H * HT + (i * 8 + wave) * 8 * BK), 16, 0, 0);
        if constexpr (!NOEPI) staged_epilogue_next0<EPI, TR>(g, acc, m0, n0, wm, wn, (char*)smem, tid);
        return;
    }
    if constexpr (NOEPI) {
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
        if (t == 1234.5f) ((float*)g.C)[tid] = t;  // keeps the loop live
    } else {
        staged_epilogue<EPI, true, TR>(g, acc, m0, n0, wm, wn, (char*)smem, tid);
    }
}

// Persistent (launch8p; OSW_GEMM_PERSIST=0: one workgroup per tile): one workgroup per CU
// looping over tiles; workgroup b runs virtual ids b, b + grid, ... (grid a multiple of 8,
// so every id of a workgroup maps to its own XCD's contiguous tile run, as in the
// one-tile-per-workgroup grid).  No encoder
// workgroups then wait in the dispatcher, where they delayed another lane's decoder
// dispatches by 17-30 us each; every decoder kernel of a greedy step must
// then fit beside an encoder workgroup (<= 30 KiB of LDS, <= 80 VGPRs); the 64-row logits
// GEMM (80 KiB) does not.  4832 vs 4789 audio-s/s (12 steps, two runs each).
// DBG (debug variants): 1 no epilogue (9: main-loop time alone), 2 the accumulators not
// transposed (the round-3 fp16 epilogues; 12, 13)
template <int EPI, int DBG = 0>
__global__ __launch_bounds__(GNT, 1) void gemm8p_kernel(GemmArgs g) {
    extern __shared__ __attribute__((aligned(16))) h16 smem[];  // [2][A0 A1 W0 W1][128*64]
    const int nwg = ((g.N + GB - 1) / GB) * ((g.M + GB - 1) / GB);
    // next0 (g.kc bit, see launch8p): the next tile's first K-tile is staged before this
    // tile's epilogue (needs an even K-tile count: the last K-tile then sits in buffer 1)
    const bool next0 = g.kc == 1 && (g.K / BK) % 2 == 0;
    bool pre0 = false;
    for (int vb = blockIdx.x; vb < nwg; vb += gridDim.x) {
        // the thread id passes through an opaque move each tile, so nothing derived from it
        // (fragment offsets, staging addresses) is hoisted out of the loop and kept live
        // across tiles: the one-tile body already needs ~206 VGPRs (hoisted: 256 + spills)
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const int nxt = next0 && vb + (int)gridDim.x < nwg ? vb + (int)gridDim.x : -1;
        gemm8p_tile<EPI, DBG>(g, vb, smem, tid, pre0, nxt);
        pre0 = nxt >= 0;
        if (!pre0) __syncthreads();  // the epilogue's LDS image is the next tile's operand ring
    }
}

// The persistent encoder GEMMs' grid (launch8p, launch8h): one workgroup per CU, or 3/4 of
// the CUs (a multiple of the 8 XCDs) while sibling lanes have calls in flight, so the other
// quarter never holds an encoder workgroup and another lane's decoder kernels run there at
// full occupancy (256 CUs: 192 workgroups, 4768 -> 4872 audio-s/s; 224: 4864, 160: 4855,
// measured).  OSW_GEMM_GRID=n: at most n workgroups while the CUs are shared;
// OSW_GEMM_PERSIST=0: no cap (one workgroup per tile).
int grid8(const GemmArgs& g) {
    static const int cus = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return 256;
        return n;
    }();
    static const bool per_tile = [] {
        const char* e = std::getenv("OSW_GEMM_PERSIST");
        return e && e[0] == '0';
    }();
    static const int shared_cap = [] {
        if (const char* gg = std::getenv("OSW_GEMM_GRID")) return std::max(8, std::min(cus, atoi(gg)) / 8 * 8);
        return std::max(8, cus * 3 / 4 / 8 * 8);
    }();
    return per_tile ? 1 << 30 : std::max(8, g.share_cus ? shared_cap : cus);
}

template <int EPI, int DBG = 0>
void launch8p(const GemmArgs& g0, hipStream_t s) {
    constexpr int lds = EPI_LDS > 8 * HT * 2 ? EPI_LDS : 8 * HT * 2;
    set_lds_once((const void*)gemm8p_kernel<EPI, DBG>, lds);
    GemmArgs g = g0;
    g.band = choose_band(g);
    // the next tile's first K-tile staged during the epilogue.  Round 3: only the head-major
    // qkv epilogue gained (1054 -> 1027 us per launch at 64 windows); the fp32 epilogues in
    // four 64-row passes (o, fc2: 886 -> 956 us) and the GELU one (1485 -> 1535 us) lost.
    // Round 6, after the epilogue work: the GELU one gains (1301 -> 1289 us), the head-major
    // one no longer does (930 without vs 940 with), the fp32 ones still lose (751 -> 779 us)
    // (profiles/r06_z_next0_ab.txt).  OSW_GEMM_NEXT0=0: never, =1: every epilogue.
    static const int next0_env = [] {
        const char* e = std::getenv("OSW_GEMM_NEXT0");
        return e ? (e[0] == '1' ? 1 : 0) : -1;
    }();
    const bool next0 = next0_env < 0 ? EPI == EPI_F16_GELU : next0_env == 1;
    g.kc = next0 ? 1 : 0;  // (kc is unused by the 8-phase kernel otherwise)
    const int nwg = ((g.N + GB - 1) / GB) * ((g.M + GB - 1) / GB);
    gemm8p_kernel<EPI, DBG><<<std::min(nwg, grid8(g)), GNT, lds, s>>>(g);
}

// Half-width tile (256 x 128 x 64) for the encoder at one to a few windows, where the 256²
// tile leaves CUs idle (qkv at one window: 90 tiles on 256 CUs) or runs a second, mostly
// empty round (fc2 at four windows: 120 tiles of 4x the K).  Same 8 waves in two groups one
// barrier apart and the same per-wave accumulator layout as gemm8p_tile restricted to the
// W0 half (rows {0,128} + wm*64 + [0,64), cols wn*32 + [0,32)), so every output element is
// the same MFMA chain over K in the same order as in the other tiles: identical results.
// Two phases per K-tile — 1: quadrant (0,0) from A0 + W0, 2: quadrant (1,0) from A1 with
// W0's fragments kept in registers — and a 3-slot ring of {A0, A1, W0} (144 KiB) so a
// K-tile is staged two tiles ahead: phase 1 of tile t stages A0(t+2), W0(t+2) (their slots'
// last reads were phase 1 of t-1, two phases back), phase 2 stages A1(t+2); each half-tile
// is waited for in the phase before its first read (three phases after its issue).  Persistent like
// gemm8p_kernel (one workgroup per CU looping over tiles).
constexpr int H8_SLOTS = 3, H8_LDS = H8_SLOTS * 3 * HT * 2;  // 147456 B
static_assert(H8_LDS >= EPI_LDS, "the epilogue image fits the ring");

template <int EPI, int DBG>
__device__ __forceinline__ void gemm8h_tile(const GemmArgs& g, int bid, h16* smem, int tid) {
    const int wave = tid >> 6, lane = tid & 63;
    constexpr bool TR = EPI == EPI_F16 || EPI == EPI_F16_GELU;
    int m0, n0;
    tile8p_origin<128>(g, bid, m0, n0);
    const h16* src[3][2];  // half-tiles 0: A0, 1: A1, 2: W0 (src8p's numbering)
#pragma unroll
    for (int H = 0; H < 3; ++H)
#pragma unroll
        for (int i = 0; i < 2; ++i) src[H][i] = src8p(g, m0, n0, H, i, wave, lane);
    auto stage = [&](int H, int t) {
        h16* base = smem + ((t % H8_SLOTS) * 3 + H) * HT;
#pragma unroll
        for (int i = 0; i < 2; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(src[H][i] + t * BK),
                                             (OSW_LDS void*)(base + (i * 8 + wave) * 8 * BK), 16, 0, 0);
    };
    const int wm = wave >> 2, wn = wave & 3;
    const int li = lane & 15, lc = lane >> 4;
    const int aoff0 = (wm * 64 + li) * BK + swz(wm * 64 + li, lc) * 8;
    const int aoff1 = (wm * 64 + li) * BK + swz(wm * 64 + li, 4 + lc) * 8;
    const int boff0 = (wn * 32 + li) * BK + swz(wn * 32 + li, lc) * 8;
    const int boff1 = (wn * 32 + li) * BK + swz(wn * 32 + li, 4 + lc) * 8;
    f32x4 acc[8][4];  // blocks ni < 2 only (the epilogue's TN = 128 form reads no others)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    h16x8 af[4][2], bf[2][2];
    auto read_a = [&](const h16* hb) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
            af[mt][0] = *(const h16x8*)&hb[aoff0 + mt * 16 * BK];
            af[mt][1] = *(const h16x8*)&hb[aoff1 + mt * 16 * BK];
        }
    };
    auto read_b = [&](const h16* hb) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
            bf[nt][0] = *(const h16x8*)&hb[boff0 + nt * 16 * BK];
            bf[nt][1] = *(const h16x8*)&hb[boff1 + nt * 16 * BK];
        }
    };
    auto barrier = [] {
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    auto mfma = [&](int a) {  // quadrant (a, 0), the 8-phase kernel's MFMA order
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {
                f32x4 c = acc[a * 4 + mt][nt];
                if constexpr (TR) {
                    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[nt][0], af[mt][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[nt][1], af[mt][1], c, 0, 0, 0);
                } else {
                    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[mt][0], bf[nt][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[mt][1], bf[nt][1], c, 0, 0, 0);
                }
                acc[a * 4 + mt][nt] = c;
            }
        __builtin_amdgcn_s_setprio(0);
    };
    const int nk = g.K / BK;
    // prologue: tiles 0 and 1 (issue order A0 W0 A1), tile 0 retired
    stage(0, 0);
    stage(2, 0);
    stage(1, 0);
    // (each half-tile is retired by itself in the phase before the one that reads it: A0, W0
    // of tile t+1 in phase 2 of tile t, A1 of tile t in phase 1 of tile t, so every half-tile
    // has three phases from issue to wait)
    if (nk > 1) {
        stage(0, 1);
        stage(2, 1);
        stage(1, 1);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // A0, W0 of tile 0
    } else {
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    }
    barrier();
    if (__builtin_amdgcn_readfirstlane(wave) >= 4) barrier();  // group 1 runs one barrier behind group 0
    for (int t = 0; t < nk; ++t) {
        const h16* buf = smem + (t % H8_SLOTS) * 3 * HT;
        const bool n1 = t + 1 < nk, n2 = t + 2 < nk;
        // phase 1: quadrant (0,0) from A0, W0; retire A1 of tile t
        if (n2) {
            stage(0, t + 2);
            stage(2, t + 2);
            asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
        } else if (n1) {
            asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        read_a(buf + 0 * HT);
        read_b(buf + 2 * HT);
        barrier();
        mfma(0);
        barrier();
        // phase 2: quadrant (1,0) from A1 (W0's fragments still in registers); retire A0, W0
        // of tile t+1
        if (n2) {
            stage(1, t + 2);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else if (n1) {
            asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        }
        read_a(buf + 1 * HT);
        barrier();
        mfma(1);
        barrier();
    }
    if (__builtin_amdgcn_readfirstlane(wave) < 4) barrier();
    if constexpr (DBG == 1) {
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
        if (t == 1234.5f) ((float*)g.C)[tid] = t;  // keeps the loop live
    } else {
        staged_epilogue<EPI, true, TR, 128>(g, acc, m0, n0, wm, wn, (char*)smem, tid);
    }
}

template <int EPI, int DBG = 0>
__global__ __launch_bounds__(GNT, 1) void gemm8h_kernel(GemmArgs g) {
    extern __shared__ __attribute__((aligned(16))) h16 smem[];  // [3][A0 A1 W0][128*64]
    const int nwg = ((g.N + 127) / 128) * ((g.M + GB - 1) / GB);
    for (int vb = blockIdx.x; vb < nwg; vb += gridDim.x) {
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));  // nothing derived from it is kept live across tiles
        gemm8h_tile<EPI, DBG>(g, vb, smem, tid);
        __syncthreads();  // the epilogue's LDS image is the next tile's operand ring
    }
}

// The half-width tile for few-window encoder GEMMs (profiles/r06_s2b_small_gemm.jsonl: every
// tile variant on the five encoder shapes at 1-4 windows).  A half tile costs about half a
// 256² tile, so with G workgroups the two grids take ceil(T/G) and ½·ceil(2T/G) tile rounds:
// the half tile where that is fewer (three and four windows: a 1.05-1.4-round 256² grid
// becomes 1.5 rounds' worth; the out-projection and fc2 at 3-4 windows fill one round),
// from 90 256² tiles (below that the 64 / 128 tiles' 2-8x the workgroups win: the
// out-projection and fc2 at one or two windows) up to 512 (the 64-window batches keep the
// tuned 8-phase grid and its 32 KiB of LDS left for other lanes' decoders: the half tile's
// 3-slot ring takes 144 KiB).  OSW_GEMM_HALF=0 turns it off (A/B switch).
bool use_half_tile(const GemmArgs& g, int64_t t8) {
    static const bool on = [] {
        const char* e = std::getenv("OSW_GEMM_HALF");
        return !(e && e[0] == '0');
    }();
    if (!on || g.A_lo || g.kc != 0 || g.N % 8 != 0 || t8 < 90 || t8 >= 512) return false;
    // below 180 256² tiles the alternative is the 64 / 128 family, whose fp16 epilogues
    // measured as fast at one window in the whole encoder (5.86 vs 5.93 ms, r06_s2c): the
    // half tile there only for the fp32 (residual) outputs, the out-projection and fc2
    if (t8 < 180 && g.epi != EPI_F32_RESID && g.epi != EPI_F32) return false;
    const int64_t G = grid8(g), th = (int64_t)((g.N + 127) / 128) * ((g.M + GB - 1) / GB);
    return ((th + G - 1) / G) < 2 * ((t8 + G - 1) / G);
}

template <int EPI, int DBG = 0>
void launch8h(const GemmArgs& g0, hipStream_t s) {
    set_lds_once((const void*)gemm8h_kernel<EPI, DBG>, H8_LDS);
    GemmArgs g = g0;
    g.band = choose_band(g, 128);
    const int nwg = ((g.N + 127) / 128) * ((g.M + GB - 1) / GB);
    gemm8h_kernel<EPI, DBG><<<std::min(nwg, grid8(g)), GNT, H8_LDS, s>>>(g);
}


template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    // s_waitcnt vmcnt(N) with expcnt/lgkmcnt left at their maxima (gfx9 encoding)
    static_assert(N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// ---------------------------------------------------------------------------
// Mid-M encoder GEMM (one to a few windows: 1500-12000 rows): 128x128x64 tiles, 4 waves
// of 64x64, and a 4-slot LDS ring (128 KiB, one workgroup per CU) that keeps three K
// tiles in flight.  The double-buffered 128 tile waited one load round trip per K step
// (fc1 at 4 windows: ~2.3 us per 64-deep step, 18 % of the CU's MFMA rate); the 64 tile
// hides the latency but moves 2x the operand bytes per flop.  Counted vmcnt + raw
// s_barrier as in gemm64_ring_kernel.  Tiles are dealt XCD-contiguously, each XCD's run
// walking down M for one column block (its weight panel stays L2-hot).  The output
// leaves through an LDS image of the tile (16-B stores, 2 KiB per wave-instruction).
// Every output element is the same MFMA chain over K in the same order as in the other
// tile sizes: identical results.
constexpr int R128_NS = 4, R128_SLOT = 2 * 128 * BK;                   // halfs per ring slot
constexpr int R128_LDS = R128_NS * R128_SLOT * 2;                      // 131072 B

template <int EPI>
__global__ __launch_bounds__(NTHR, 1) void gemm128_ring_kernel(GemmArgs g) {
    constexpr int TM = 128, PW = 4, FT = 4, WT = 64;
    extern __shared__ __attribute__((aligned(16))) h16 smem[];  // [NS][A|W][128*64]
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int ntm = (g.M + TM - 1) / TM, ntn = (g.N + TM - 1) / TM, nwg = ntm * ntn;
    const int bid = blockIdx.x, q = nwg / 8, r8 = nwg % 8, xcd = bid % 8;
    const int v = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + bid / 8;
    const int m0 = (v % ntm) * TM, n0 = (v / ntm) * TM;
    const h16* asrc[PW];
    const h16* wsrc[PW];
#pragma unroll
    for (int i = 0; i < PW; ++i) {
        const int r = (i * 4 + wave) * 8 + (lane >> 3);
        const int c = swz(r, lane & 7);
        asrc[i] = grp_row(g.A, min(m0 + r, g.M - 1), g.a_grp_rows, g.a_grp_stride, g.lda) + c * 8;
        wsrc[i] = g.W + (int64_t)min(n0 + r, g.N - 1) * g.ldw + c * 8;
    }
    auto stage = [&](int slot, int k0) {
        h16* base = smem + slot * R128_SLOT;
#pragma unroll
        for (int i = 0; i < PW; ++i) {
            __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + k0), (OSW_LDS void*)(base + (i * 4 + wave) * 8 * BK),
                                             16, 0, 0);
            __builtin_amdgcn_global_load_lds((const void*)(wsrc[i] + k0),
                                             (OSW_LDS void*)(base + TM * BK + (i * 4 + wave) * 8 * BK), 16, 0, 0);
        }
    };
    const int wm = wave >> 1, wn = wave & 1;
    f32x4 acc[FT][FT];
#pragma unroll
    for (int i = 0; i < FT; ++i)
#pragma unroll
        for (int j = 0; j < FT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nk = g.K / BK;
#pragma unroll
    for (int s = 0; s < R128_NS - 1; ++s)
        if (s < nk) stage(s, s * BK);
    for (int kt = 0; kt < nk; ++kt) {
        // tile kt has landed once at most min(NS-2, nk-1-kt) younger tiles are in flight
        const int ahead = min(R128_NS - 2, nk - 1 - kt);
        if (ahead >= 2) wait_vmcnt<2 * 2 * PW>();
        else if (ahead == 1) wait_vmcnt<2 * PW>();
        else wait_vmcnt<0>();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every wave's pieces of tile kt landed; slot (kt-1) % NS is free
        asm volatile("" ::: "memory");
        if (kt + R128_NS - 1 < nk) stage((kt + R128_NS - 1) % R128_NS, (kt + R128_NS - 1) * BK);
        const h16* la = smem + (kt % R128_NS) * R128_SLOT;
        const h16* lw = la + TM * BK;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int c = ks * 4 + (lane >> 4);
            h16x8 a[FT], b[FT];
#pragma unroll
            for (int mi = 0; mi < FT; ++mi) {
                const int row = wm * WT + mi * 16 + (lane & 15);
                a[mi] = *(const h16x8*)&la[row * BK + swz(row, c) * 8];
            }
#pragma unroll
            for (int ni = 0; ni < FT; ++ni) {
                const int row = wn * WT + ni * 16 + (lane & 15);
                b[ni] = *(const h16x8*)&lw[row * BK + swz(row, c) * 8];
            }
#pragma unroll
            for (int mi = 0; mi < FT; ++mi)
#pragma unroll
                for (int ni = 0; ni < FT; ++ni)
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
        }
    }
    // epilogue through an LDS image of the tile (the ring is free once every wave is past
    // its last fragment read)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if constexpr (EPI != EPI_F32) {
        staged_epilogue_sq<EPI, TM>(g, acc, m0, n0, wm, wn, smem, threadIdx.x);
    } else {  // (debug entry only) plain fp32 tile
#pragma unroll
        for (int mi = 0; mi < FT; ++mi)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int m = m0 + wm * WT + mi * 16 + (lane >> 4) * 4 + i;
                if (m >= g.M) continue;
#pragma unroll
                for (int ni = 0; ni < FT; ++ni) {
                    const int n = n0 + wn * WT + ni * 16 + (lane & 15);
                    if (n < g.N) ((float*)g.C)[c_row(g, m) + n] =
                        g.bias ? acc[mi][ni][i] + g.bias[n] : acc[mi][ni][i];
                }
            }
    }
}

template <int EPI>
void launch_ring128(const GemmArgs& g, hipStream_t s) {
    set_lds_once((const void*)gemm128_ring_kernel<EPI>, R128_LDS);
    const int nwg = ((g.N + 127) / 128) * ((g.M + 127) / 128);
    gemm128_ring_kernel<EPI><<<nwg, NTHR, R128_LDS, s>>>(g);
}

// ---------------------------------------------------------------------------
// Skinny GEMM for the decoder (M <= 64 rows = windows in the batch): weight-
// bandwidth bound, so the grid is split over N (64 columns per workgroup, 16 per
// wave) AND over K (ksplit partial slabs, reduced deterministically by a second
// kernel that also applies the epilogue).  Operands go straight to VGPRs
// (no LDS: nothing is shared between waves but the tiny, L2-resident A).

// Small-M encoder GEMM (one or a few windows): 64x64 tiles (4 waves of 32x32) with a
// 4-slot LDS ring that keeps three K tiles in flight.  A 64-tile K step is only 8 MFMAs
// per wave, far shorter than the load latency, so the double-buffered gemm_kernel<.., 64>
// waited ~one HBM round trip per K step (fc2 at 1500 rows: 80 steps, ~70 us).  Counted
// vmcnt + raw s_barrier (a __syncthreads would drain every LDS-DMA in flight).  The
// MFMA chain of every output element is gemm_kernel's, in the same K order: identical
// results.
constexpr int R64_NS = 4;
template <int EPI>
__global__ __launch_bounds__(NTHR, 2) void gemm64_ring_kernel(GemmArgs g) {
    constexpr int TM = 64, PW = 2, FT = 2, WT = 32;
    __shared__ __attribute__((aligned(16))) h16 lds[R64_NS][2][TM * BK];  // 64 KiB
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n0 = blockIdx.x * TM, m0 = blockIdx.y * TM;
    const h16* asrc[PW];
    const h16* wsrc[PW];
#pragma unroll
    for (int i = 0; i < PW; ++i) {
        const int r = (i * 4 + wave) * 8 + (lane >> 3);
        const int c = swz(r, lane & 7);
        asrc[i] = grp_row(g.A, min(m0 + r, g.M - 1), g.a_grp_rows, g.a_grp_stride, g.lda) + c * 8;
        wsrc[i] = g.W + (int64_t)min(n0 + r, g.N - 1) * g.ldw + c * 8;
    }
    auto stage = [&](int slot, int k0) {
#pragma unroll
        for (int i = 0; i < PW; ++i) {
            __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + k0), (OSW_LDS void*)&lds[slot][0][(i * 4 + wave) * 8 * BK],
                                             16, 0, 0);
            __builtin_amdgcn_global_load_lds((const void*)(wsrc[i] + k0), (OSW_LDS void*)&lds[slot][1][(i * 4 + wave) * 8 * BK],
                                             16, 0, 0);
        }
    };
    const int wm = wave >> 1, wn = wave & 1;
    f32x4 acc[FT][FT];
#pragma unroll
    for (int i = 0; i < FT; ++i)
#pragma unroll
        for (int j = 0; j < FT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nk = g.K / BK;
#pragma unroll
    for (int s = 0; s < R64_NS - 1; ++s)
        if (s < nk) stage(s, s * BK);
    for (int kt = 0; kt < nk; ++kt) {
        // tile kt has landed once at most min(NS-2, nk-1-kt) younger tiles are in flight
        const int ahead = min(R64_NS - 2, nk - 1 - kt);
        if (ahead >= 2) wait_vmcnt<2 * 2 * PW>();
        else if (ahead == 1) wait_vmcnt<2 * PW>();
        else wait_vmcnt<0>();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every wave's pieces of tile kt landed; slot (kt-1) % NS is free
        asm volatile("" ::: "memory");
        if (kt + R64_NS - 1 < nk) stage((kt + R64_NS - 1) % R64_NS, (kt + R64_NS - 1) * BK);
        const h16* la = lds[kt % R64_NS][0];
        const h16* lw = lds[kt % R64_NS][1];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int c = ks * 4 + (lane >> 4);
            h16x8 a[FT], b[FT];
#pragma unroll
            for (int mi = 0; mi < FT; ++mi) {
                const int row = wm * WT + mi * 16 + (lane & 15);
                a[mi] = *(const h16x8*)&la[row * BK + swz(row, c) * 8];
            }
#pragma unroll
            for (int ni = 0; ni < FT; ++ni) {
                const int row = wn * WT + ni * 16 + (lane & 15);
                b[ni] = *(const h16x8*)&lw[row * BK + swz(row, c) * 8];
            }
#pragma unroll
            for (int mi = 0; mi < FT; ++mi)
#pragma unroll
                for (int ni = 0; ni < FT; ++ni)
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
        }
    }
    if constexpr (EPI != EPI_F32) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __syncthreads();  // every wave past its last fragment read: the ring holds the image
        staged_epilogue_sq<EPI, TM>(g, acc, m0, n0, wm, wn, &lds[0][0][0], threadIdx.x);
        return;
    }
#pragma unroll
    for (int mi = 0; mi < FT; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int m = m0 + wm * WT + mi * 16 + (lane >> 4) * 4 + i;
            if (m >= g.M) continue;
#pragma unroll
            for (int ni = 0; ni < FT; ++ni) {
                const int n = n0 + wn * WT + ni * 16 + (lane & 15);
                if (n >= g.N) continue;
                if constexpr (EPI == EPI_F32) {
                    const float v = g.bias ? acc[mi][ni][i] + g.bias[n] : acc[mi][ni][i];
                    const int64_t grp = fast_div(m, g.c_grp_rows), r = m - grp * g.c_grp_rows;
                    __hip_atomic_store((float*)g.C + grp * g.c_grp_stride + r * g.ldc + n, v, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                } else
                    store_one<EPI>(g, m, n, acc[mi][ni][i]);
            }
        }
}

__device__ __forceinline__ void sel_merge(SelPart& r, const SelPart& q) {
    lse_merge(r.m_all, r.s_all, q.m_all, q.s_all);
    lse_merge(r.m_ts, r.s_ts, q.m_ts, q.s_ts);
    const ArgMax A = amax(ArgMax{r.v_all, r.i_all}, ArgMax{q.v_all, q.i_all});
    const ArgMax X = amax(ArgMax{r.v_text, r.i_text}, ArgMax{q.v_text, q.i_text});
    const ArgMax T = amax(ArgMax{r.v_ts, r.i_ts}, ArgMax{q.v_ts, q.i_ts});
    r.v_all = A.v; r.i_all = A.i; r.v_text = X.v; r.i_text = X.i; r.v_ts = T.v; r.i_ts = T.i;
}

__device__ __forceinline__ SelPart sel_xor(const SelPart& r, int o) {
    SelPart q;
    switch (o) {  // xor_lane needs a compile-time offset
#define OSW_SX(O) case O: q = SelPart{xor_lane<O>(r.m_all), xor_lane<O>(r.s_all), xor_lane<O>(r.m_ts), \
                                      xor_lane<O>(r.s_ts), xor_lane<O>(r.v_all), xor_lane<O>(r.v_text), \
                                      xor_lane<O>(r.v_ts), xor_lane<O>(r.i_all), xor_lane<O>(r.i_text), \
                                      xor_lane<O>(r.i_ts)}; break;
        OSW_SX(32) OSW_SX(16) OSW_SX(8) OSW_SX(4) OSW_SX(2) default: OSW_SX(1)
#undef OSW_SX
    }
    return q;
}

// A workgroup's SelPart over 64 lanes x 4 waves (fixed merge pattern), in thread 0.
__device__ __forceinline__ SelPart sel_block_merge(SelPart r, SelPart* wp) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const SelPart q = sel_xor(r, o);
        sel_merge(r, q);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) wp[w] = r;
    __syncthreads();
    SelPart t = wp[0];
    for (int i = 1; i < 4; ++i) sel_merge(t, wp[i]);
    return t;
}

// The selection of select_kernel (greedy, one row) on the logits this workgroup just
// computed: lane `valid` holds logit x of vocabulary entry `col`.  Entries are folded
// into the slice statistics exactly as select_partial_body does; the workgroup's record
// goes to parts[blockIdx.x] and the last workgroup to arrive merges all records in
// workgroup order, finalises the row and advances the step counter.
// The step counter, the row's state and the lane's suppress-mask word are loaded when the
// workgroup starts (SelPre), in the shadow of the weight stream, not after the GEMM: two
// dependent round trips fewer at every workgroup's end (the last arriver writes them only
// after every workgroup has taken its ticket, i.e. after every workgroup loaded them).
struct SelPre {
    int step;
    SelState s;
    unsigned supw;
};
__device__ __forceinline__ SelPre sel_preload(const SelFuse& F, int col) {
    SelPre q;
    q.step = *F.pos;
    q.s = F.st[0];
    q.supw = F.supmask[min(col, F.P.V - 1) >> 5];
    return q;
}

__device__ __forceinline__ void fused_select_row(float x, int col, bool valid, const SelFuse& F, const SelPre& pre) {
    __shared__ SelPart wp[4];
    __shared__ int last;
    const SelParams& P = F.P;
    const int step = pre.step;
    const SelState s = pre.s;
    const int mode = sel_mode(P, step, s);
    const SelPart id{-INFINITY, 0.f, -INFINITY, 0.f, -INFINITY, -INFINITY, -INFINITY, 0x7fffffff, 0x7fffffff,
                     0x7fffffff};
    SelPart r = id;
    if (valid && (mode == SEL_SOT || mode == SEL_SAMPLE)) {
        ArgMax a_all{-INFINITY, 0x7fffffff}, a_text{-INFINITY, 0x7fffffff}, a_ts{-INFINITY, 0x7fffffff};
        const int v = col;
        if (mode == SEL_SOT) {
            lse_add(r.m_all, r.s_all, x);
            if (v >= P.first_lang && v < P.first_lang + P.n_langs) a_text = ArgMax{x, v};
        } else if (!tok_masked_w(P, row_rules(P, s), pre.supw, v)) {
            lse_add(r.m_all, r.s_all, x);
            a_all = ArgMax{x, v};
            if (v >= P.tb) {
                lse_add(r.m_ts, r.s_ts, x);
                a_ts = ArgMax{x, v};
            } else {
                a_text = ArgMax{x, v};
            }
        }
        r.v_all = a_all.v; r.i_all = a_all.i; r.v_text = a_text.v; r.i_text = a_text.i; r.v_ts = a_ts.v; r.i_ts = a_ts.i;
    }
    SelPart* parts = (SelPart*)F.parts;
    const int nwg = gridDim.x;
    r = sel_block_merge(r, wp);
    if (threadIdx.x == 0) {
        store_part(parts + blockIdx.x, r);
        __builtin_amdgcn_s_waitcnt(0);  // the record is complete at device scope before the ticket
        last = __hip_atomic_fetch_add(F.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nwg - 1;
        if (last) __hip_atomic_store(F.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last) return;
    // every record this thread merges is loaded before any is merged: one round trip for
    // the <= 4 records per thread (811 workgroups at turbo), not one per record
    constexpr int RPT = 4;
    SelPart rec[RPT];
#pragma unroll
    for (int j = 0; j < RPT; ++j) rec[j] = load_part(parts + min((int)threadIdx.x + 256 * j, nwg - 1));
    SelPart t = id;
#pragma unroll
    for (int j = 0; j < RPT; ++j)
        if ((int)threadIdx.x + 256 * j < nwg) sel_merge(t, rec[j]);
    for (int i = threadIdx.x + 256 * RPT; i < nwg; i += 256) sel_merge(t, load_part(parts + i));
    __syncthreads();  // wp is reused
    t = sel_block_merge(t, wp);
    if (threadIdx.x != 0) return;
    // the logits the finaliser reads back (no-speech prob, an <|endoftext|> log-prob) were
    // stored by other workgroups of this launch: write-through stores, device-scope loads
    select_finalize<true>(F.logits, P, step, F.prompt, [&] { return t; }, F.st, F.cur_tok, F.tokens, F.max_tokens,
                          0);
    __builtin_amdgcn_s_waitcnt(0);
    __hip_atomic_store(F.pos, step + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int MT, bool DIRECT, int EPI, bool LO, int PRO = PRO_NONE, bool SEL = false, int TAIL = TAIL_NONE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SEL ? 4 : 1, 8))) void gemm_skinny_kernel(GemmArgs g, int kc, float* __restrict__ part, ProArgs pa) {
    // Workgroup = 64 columns x one kc-deep K range; wave = 16 columns.  The
    // activation rows (M <= 64) of each CKK-deep K chunk are staged ONCE per
    // workgroup into LDS by global_load_lds (row-XOR swizzle on the 16-B chunk ->
    // conflict-free ds_read_b128), instead of every wave re-reading them from L2
    // (4x the weight bytes at M = 64).  Weights stream straight to VGPRs, CK x 16 B
    // per lane per chunk, the next chunk's loads issued before the current chunk's
    // MFMAs (two register sets, manual 2x unroll).  Loads are unconditional (clamped
    // addresses for a short last chunk) so hipcc never branches around them.
    // LO: a second image holds the activations' lo halves (GemmArgs::A_lo); every
    // weight fragment feeds two MFMAs (hi, then lo) into one accumulator.  At > 32
    // rows the chunk is 128 k so both images still fit 64 KB (2 workgroups per CU).
    // PRO (<= 8 rows, hi/lo): the activation rows are not loaded but built by the
    // workgroup from the producer's split-K slabs (resln.h) into an LDS image Ap while
    // the first weight chunk is in flight: residual+LayerNorm of the whole row (PRO_RESLN)
    // or the GELU reduce of this workgroup's K range (PRO_GELU).  The MFMA order is the
    // plain kernel's, so both paths give identical results.
    static_assert(PRO == PRO_NONE || (MT == 1 && LO), "the prologue serves <= 8 hi/lo rows");
    // k32 steps per chunk; >= 32 hi/lo rows use 64-deep chunks: the two A buffers of 32
    // rows are then 16 KiB, so a workgroup fits beside another lane's encoder GEMM
    // workgroup (which leaves 30 KiB of the CU's LDS free, tools/coresidency_probe.hip)
    // (48 hi/lo rows: 128-deep chunks, so the 4 waves' 1-KiB staging pieces cover all 48
    // rows; a 64-deep chunk stages 32 rows per round and would leave rows 32-47 unstaged.
    // Not reachable from the launchers, which group hi/lo rows by 32; kept valid anyway.)
    // 16-row hi/lo groups (2..16 decoder rows: beam 5 of one to three windows, greedy
    // batches) stream 128-deep chunks: 16 KiB of LDS, so the workgroup fits beside another
    // lane's 128-KiB encoder workgroup (<= 30 KiB free) instead of waiting for its tile to
    // retire; the fused batch-1 forms (PRO) keep 256-deep chunks
    constexpr int CK = (LO && MT >= 2) ? (MT == 3 ? 4 : 2) : (LO && PRO == PRO_NONE) ? OSW_SKINNY_CK1 : 8;
    constexpr int CKK = CK * 32;                 // k per chunk
    constexpr int CPR = CKK / 8;                 // 16-B pieces of one row per chunk
    constexpr int RPP = 64 / CPR;                // rows per 1-KiB glds wave-instruction
    constexpr int SWM = (CPR < 16 ? CPR : 16) - 1;  // XOR swizzle of the 16-B chunk by row, within the row
    constexpr int ROWS = MT * 16;
    constexpr int NIMG = LO ? 2 : 1;
    constexpr int APIECES = ROWS / RPP / 4;      // glds per wave per image per chunk
    static_assert(PRO != PRO_NONE || APIECES * 4 * RPP == ROWS, "the staging pieces cover every row exactly once");
    __shared__ __attribute__((aligned(16))) h16 As[PRO ? 1 : 2][NIMG][PRO ? 8 : ROWS * CKK];
    constexpr int APR = PRO == PRO_GELU ? GELU_ROWS : PRO == PRO_RESLN ? PRO_ROWS : 1;  // image rows
    constexpr int APS = PRO == PRO_GELU ? GELU_KC + 8 : PRO == PRO_RESLN ? PRO_STRIDE : 8;
    __shared__ __attribute__((aligned(16))) h16 Ap[PRO ? 2 : 1][APR][APS];
    __shared__ __attribute__((aligned(16))) float pred[PRO ? resln_scratch(PRO_ROWS, 1280) : 1];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
    if (g.pair_rows) {
        // 1-D grid: workgroup id = 8 j + xcd, j = unit * nz + row group, unit = (column
        // block, K range) numbered xcd-major: every row group of a unit on one XCD, adjacent
        const int nz = (g.M + ROWS - 1) / ROWS, gx = (g.N + 63) / 64, units = gx * (g.K / kc);
        const int j = blockIdx.x >> 3;
        const int u = (j / nz) * 8 + (blockIdx.x & 7);
        if (u >= units) return;
        bz = j % nz;
        bx = u % gx;
        by = u / gx;
    }
    const int nb = bx * 64 + wave * 16;
    const int ks = by;
    const int mb = bz * ROWS;  // row group (partial mode, M > 64: beam rows)
    const int k0 = ks * kc;
    // this lane's weights: column nb + (lane & 15), k = k0 + 8 (lane >> 4) + 32 st
    const h16* wrow;
    int wss;  // h16 per k32 step
    if (g.Wf) {
        // fragment-major copy: the wave's 16 x 32 fragment of step st is 1 KB contiguous
        // (a block past the padded N repeats the last one; its columns are discarded)
        const int blk = min(nb, ((g.N + 15) & ~15) - 16) >> 4;
        wrow = g.Wf + ((int64_t)blk * (g.K >> 5) + (k0 >> 5)) * 512 + lane * 8;
        wss = 512;
    } else {
        const int n = min(nb + (lane & 15), g.N - 1);
        wrow = g.W + (int64_t)n * g.ldw + k0 + 8 * (lane >> 4);
        wss = 32;
    }
    SelPre sel_pre{};
    if constexpr (SEL) sel_pre = sel_preload(pa.sel, nb + (lane & 15));
    const int nsteps = kc / 32;  // multiple of 4
    const int nch = (nsteps + CK - 1) / CK;

    const h16* asrc[NIMG][APIECES];
    int acl[APIECES];
#pragma unroll
    for (int i = 0; i < APIECES; ++i) {
        const int j = i * 4 + wave;
        const int row = RPP * j + lane / CPR;
        acl[i] = ((lane % CPR) ^ (row & SWM)) * 8;
        const int64_t gr = min(mb + row, g.M - 1);
        asrc[0][i] = grp_row(g.A, gr, g.a_grp_rows, g.a_grp_stride, g.lda) + k0;
        if constexpr (LO) asrc[NIMG - 1][i] = grp_row(g.A_lo, gr, g.a_grp_rows, g.a_grp_stride, g.lda) + k0;
    }
    auto stageA = [&](int buf, int c) {
        if constexpr (PRO != PRO_NONE) return;
        // a short last chunk is staged from kc-CKK so every load stays inside this K range;
        // with kc < CKK the unused tail is clamped to the range's last 16 B (values unused)
        const int kk = min(c * CKK, kc - CKK > 0 ? kc - CKK : 0);
#pragma unroll
        for (int im = 0; im < NIMG; ++im)
#pragma unroll
            for (int i = 0; i < APIECES; ++i) {
                const int j = i * 4 + wave;
                __builtin_amdgcn_global_load_lds((const void*)(asrc[im][i] + min(kk + acl[i], kc - 8)),
                                                 (OSW_LDS void*)&As[buf][im][RPP * j * CKK], 16, 0, 0);
            }
    };
    auto loadW = [&](h16x8 (&wf)[CK], int c) {
#pragma unroll
        for (int u = 0; u < CK; ++u) {
            const int st = min(c * CK + u, nsteps - 1);
            // (nt loads measured 8.1 vs 7.2 us on the projections: their weights are re-read
            // every step; nt on the logits stream alone left the batch-1 p50 unchanged)
            wf[u] = *(const h16x8*)(wrow + (int64_t)wss * st);
        }
    };
    f32x4 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int li = lane & 15, gq = lane >> 4;
    auto consume = [&](const h16x8 (&wf)[CK], int buf, int c) {
        const int steps = min(CK, nsteps - c * CK);
        // a short last chunk was staged from kc-CKK: its k32 steps sit at the end of the image
        const int shift = (c * CKK > kc - CKK && kc >= CKK) ? (c * CKK - (kc - CKK)) / 32 : 0;
#pragma unroll
        for (int u = 0; u < CK; ++u) {
            if (u >= steps) break;
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                const int row = mt * 16 + li;
                h16x8 af, al;
                if constexpr (PRO != PRO_NONE) {
                    // image column of k = k0 + c*CKK + 32u + 8gq (the whole row for RESLN, the
                    // workgroup's K range for GELU); rows past M repeat row M-1 (discarded)
                    const int r = min(row, g.M - 1);
                    const int kk = (PRO == PRO_RESLN ? k0 : 0) + c * CKK + u * 32 + gq * 8;
                    af = *(const h16x8*)&Ap[0][r][kk];
                    al = *(const h16x8*)&Ap[PRO ? 1 : 0][r][kk];
                } else {
                    const int ch = ((u + shift) * 4 + gq) ^ (row & SWM);
                    af = *(const h16x8*)&As[buf][0][row * CKK + ch * 8];
                    if constexpr (LO) al = *(const h16x8*)&As[buf][NIMG - 1][row * CKK + ch * 8];
                }
                acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, wf[u], acc[mt], 0, 0, 0);
                if constexpr (LO) acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, wf[u], acc[mt], 0, 0, 0);
            }
        }
    };
    constexpr int INFLIGHT = CK + (PRO ? 0 : NIMG * APIECES);  // one chunk's loads per lane
    // 32-row hi/lo groups stream 64-deep chunks (CK = 2): one chunk of weights ahead is
    // 8 KB in flight per workgroup, so the 32 KB of a 256-deep K range took ~4 dependent
    // HBM round trips.  With preload_w every k32 step's weights (8 x 16 B per lane, 32
    // VGPRs) is issued at the start: one round trip, the A chunks staged behind it.
    if constexpr (PRO == PRO_NONE && CK < 8) {
        constexpr int WALL = 8;
        if (g.preload_w && nsteps <= WALL) {
            constexpr int AL = NIMG * APIECES;   // LDS-DMA loads per lane per chunk
            h16x8 w[WALL];
#pragma unroll
            for (int u = 0; u < WALL; ++u) w[u] = *(const h16x8*)(wrow + (int64_t)wss * min(u, nsteps - 1));
            stageA(0, 0);
            if (nch > 1) stageA(1, 1);
#pragma unroll
            for (int c = 0; c < WALL / CK; ++c) {
                if (c >= nch) break;
                if (c + 1 < nch) wait_vmcnt<AL>();   // chunk c's A landed (and every weight load)
                else wait_vmcnt<0>();
                __builtin_amdgcn_s_barrier();
                h16x8 wf[CK];
#pragma unroll
                for (int u = 0; u < CK; ++u) wf[u] = w[c * CK + u];
                consume(wf, c & 1, c);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                if (c + 2 < nch) stageA(c & 1, c + 2);
            }
            goto store;
        }
    }
    {
    h16x8 wa[CK], wb[CK];
    loadW(wa, 0);
    stageA(0, 0);
    // the fused-selection logits GEMM (5 chunks): the second chunk goes out before the
    // prologue too (GemmArgs::preload_w), so two chunks stream while the row is normalised
    const bool wb_early = SEL && g.preload_w && nch > 1;
    if (wb_early) loadW(wb, 1);
    if constexpr (PRO == PRO_RESLN) {
        // every workgroup normalises all rows (a few KB from L2); one stores x'
        const bool wx = blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0;
        auto put = [&](int r, int c, float y) {
            const h16 h = (h16)y;
            Ap[0][r][c] = h;
            Ap[PRO ? 1 : 0][r][c] = (h16)(y - (float)h);
        };
        // all slab loads of the row in one round trip (24 covers fc2's 20 slabs)
        // (the fused-selection logits GEMM: 10 per batch, two round trips for fc2's 20 slabs,
        // so its VGPRs fit 4 workgroups per CU and its 811 workgroups run in one round)
        constexpr int KBIG = SEL ? 8 : 24;
        // (early residual loads where the VGPRs allow: not in the selecting logits GEMM, not
        // beside 24 slabs)
        if (pa.ln.ks <= 8) resln_rows<PRO_ROWS, 8, !SEL>(pa.ln, 0, g.M, wx, pred, put);
        else resln_rows<PRO_ROWS, KBIG, false>(pa.ln, 0, g.M, wx, pred, put);
        __syncthreads();
    } else if constexpr (PRO == PRO_GELU) {
        const int64_t slab = (int64_t)g.M * g.K;
        auto rows = [&](auto nr) {
            constexpr int NR = decltype(nr)::value;
            for (int j = threadIdx.x; j < kc; j += 256) {
                float y[NR];
                gelu_reduce_rows<NR>(pa.part, pa.ks, slab, pa.bias, g.M, g.K, k0 + j, y);
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const h16 h = (h16)y[r];
                    Ap[0][r][j] = h;
                    Ap[PRO ? 1 : 0][r][j] = (h16)(y[r] - (float)h);
                }
            }
        };
        if (g.M <= 1) rows(std::integral_constant<int, 1>{});
        else if (g.M <= 2) rows(std::integral_constant<int, 2>{});
        else if (g.M <= 4) rows(std::integral_constant<int, 4>{});
        else rows(std::integral_constant<int, GELU_ROWS>{});
        __syncthreads();
    }
    for (int c = 0; c < nch; c += 2) {
        if (c + 1 < nch) {
            if (!(wb_early && c == 0)) loadW(wb, c + 1);
            stageA(1, c + 1);
            wait_vmcnt<INFLIGHT>();
        } else {
            wait_vmcnt<0>();
        }
        __builtin_amdgcn_s_barrier();
        consume(wa, 0, c);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (c + 1 >= nch) break;
        if (c + 2 < nch) {
            loadW(wa, c + 2);
            stageA(0, c + 2);
            wait_vmcnt<INFLIGHT>();
        } else {
            wait_vmcnt<0>();
        }
        __builtin_amdgcn_s_barrier();
        consume(wb, 1, c + 1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }
    }
store:
    const int col = nb + li;
    if constexpr (SEL) {
        static_assert(MT == 1 && DIRECT, "the fused selection serves the batch-1 logits GEMM");
        const bool valid = gq == 0 && col < g.N;
        if (valid) __hip_atomic_store((float*)g.C + col, acc[0][0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fused_select_row(acc[0][0], col, valid, pa.sel, sel_pre);
        return;
    }
    if (col < g.N) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int m = mb + mt * 16 + gq * 4 + i;
                if (m >= g.M) continue;
                if constexpr (DIRECT) store_one<EPI>(g, m, col, acc[mt][i]);
                // slabs are written through L2 (device-scope stores): no dirty lines left for
                // the kernel-boundary write-back to drain before the consumer can start.  (Staging
                // the tile through LDS for 8-B coalesced stores, as gemm_wide_kernel does, cost
                // more in barriers than it saved: 7.7 -> 8.3 us at 64 rows, measured.)
                else __hip_atomic_store(&part[((int64_t)ks * g.M + m) * g.N + col], acc[mt][i], __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
            }
    }
    if constexpr (TAIL == TAIL_ATTN) {
        // batch-1 qkv projection (PRO_RESLN, split-K slabs): column block bx is q, k or v of
        // head bx % H; the last of a head's 3 x ks workgroups to finish runs that head's
        // self-attention (self_attn_one, the standalone kernel's function: same bits), so the
        // self-attention is not launched.  Every slab store of this workgroup is complete at
        // device scope before its ticket; the tail reads the slabs with device-scope loads.
        static_assert(!DIRECT && PRO == PRO_RESLN && !SEL && MT == 1, "the attention tail serves the batch-1 qkv GEMM");
        __shared__ int a_last;
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        const SelfAttnTail& at = pa.attn;
        const int nks = g.K / kc, hh = bx % at.H;
        if (threadIdx.x == 0) {
            int* tk = pa.tail_ticket + hh;
            a_last = __hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 3 * nks - 1;
            if (a_last) __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (!a_last) return;
        self_attn_one<true, true>(part, nks, at.bias, at.kc, at.vc, at.pos, at.H, 1, at.ctx, at.out, at.lo_off, at.st,
                                  at.pos_row, 0, hh);
    }
    if constexpr (TAIL == TAIL_GELU) {
        static_assert(!DIRECT && PRO == PRO_NONE && !SEL, "the GELU tail reduces split-K slabs");
        // the last of the block's ks workgroups reduces its 64 columns x ROWS rows; every
        // slab store of this workgroup is complete at device scope before its ticket
        __shared__ int t_last;
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        const int nz = (g.M + ROWS - 1) / ROWS, nks = g.K / kc;
        if (threadIdx.x == 0) {
            int* tk = pa.tail_ticket + bx * nz + bz;
            t_last = __hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nks - 1;
            if (t_last) __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (!t_last) return;
        // element e = r * 64 + c of the block, EPT per thread; the slabs were written by other
        // workgroups of this launch (other XCDs): device-scope loads.  Every element's loads of
        // a batch of 8 slabs are issued before any is added; the adds in gelu_reduce_one's order
        constexpr int EPT = ROWS * 64 / 256;
        const int64_t slab = (int64_t)g.M * g.N;
        int64_t off[EPT];
        float v[EPT];
        bool ok[EPT];
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
            const int e = threadIdx.x + 256 * j, m = mb + (e >> 6), n = bx * 64 + (e & 63);
            ok[j] = m < g.M && n < g.N;
            off[j] = (int64_t)min(m, g.M - 1) * g.N + min(n, g.N - 1);
            v[j] = pa.bias[min(n, g.N - 1)];
        }
        for (int k0 = 0; k0 < nks; k0 += 8) {
            float p[EPT][8];
#pragma unroll
            for (int j = 0; j < EPT; ++j)
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    p[j][q] = __hip_atomic_load(part + (int64_t)min(k0 + q, nks - 1) * slab + off[j], __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int j = 0; j < EPT; ++j)
#pragma unroll
                for (int q = 0; q < 8; ++q) v[j] += k0 + q < nks ? p[j][q] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < EPT; ++j)
            if (ok[j]) split_h16(gelu_erf(v[j]), pa.tail_y, pa.tail_y + pa.tail_lo, off[j]);
    }
}

// Wide-N GEMM for the decoder (logits: 64-row tiles x the 51866 vocabulary columns;
// beam search's > 64 rows: every projection): 64 rows x 128 columns per workgroup,
// 4 waves of 64 x 32, fp32 out written through L2 (device-scope stores) for the
// consumer kernels.  A 3-slot LDS ring keeps two 64-deep weight tiles in flight
// per workgroup (the generic 128x128 kernel keeps one and waits a full HBM round
// trip per K tile: 44.9 -> 35.8 us per logits step at 64 rows).  Grid: x = column
// tiles, y = 64-row tiles, z = split-K slabs (g.kc > 0: slab z at C + z*M*ldc, no
// bias, the projections of beam rows).
// LO (hi/lo activations, GemmArgs::A_lo): the activations come from L2 (tiny, hot),
// so their ring is only 2 slots, staged one tile ahead instead of two: 32 KB of A
// (hi + lo) + 48 KB of W = 80 KB, 2 workgroups per CU as without LO (the 96 KB
// 3-slot version held one per CU and ran the 406 logits tiles in two rounds:
// 58.8 us per step).
constexpr int WBM = 64, WBN = 128, WSL = 3;
// WN = 256 (the vocabulary logits, N >= 16384, no split-K): 8 waves and a 64 x 256 tile, one
// workgroup per CU (128 KiB of dynamic LDS).  Per 64-deep K step a workgroup stages
// (64 rows of A, hi + lo) + WN rows of W: 256 columns stage 25 % fewer bytes per MAC than
// 128 (at 320 beam rows the 133 MB matrix is staged 5 times either way, the activations
// 203 instead of 406 times).  Same MFMA chain per output element: identical results.
template <int WN>
constexpr int wide_lds(bool lo) { return (lo ? 2 * 2 : WSL) * WBM * BK * 2 + WSL * WN * BK * 2; }

template <bool LO, int WN = WBN>
__global__ __launch_bounds__(WN * 2, WN == WBN ? 2 : 1) void gemm_wide_kernel(GemmArgs g) {
    constexpr int NIMG = LO ? 2 : 1;
    constexpr int ASL = LO ? 2 : WSL;  // A ring slots
    constexpr int NW = WN / 32, NT = 64 * NW;  // waves, threads
    constexpr int GA = 8 / NW;                 // A staging groups (8 rows x 64 k) per wave and image
    h16* la;  // [ASL][NIMG][WBM * BK]
    h16* lw;  // [WSL][WN * BK]
    if constexpr (WN == WBN) {
        __shared__ __attribute__((aligned(16))) h16 sa[ASL][NIMG][WBM * BK];
        __shared__ __attribute__((aligned(16))) h16 sw[WSL][WN * BK];
        la = &sa[0][0][0];
        lw = &sw[0][0];
    } else {
        extern __shared__ __attribute__((aligned(16))) h16 smem[];
        la = smem;
        lw = smem + ASL * NIMG * WBM * BK;
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n0 = blockIdx.x * WN, m0 = blockIdx.y * WBM;
    const int kc = g.kc > 0 ? g.kc : g.K, kbeg = blockIdx.z * kc;
    // staging: one wave-instruction fills 8 rows x 64 k (1 KiB); A 8 groups (GA per
    // wave) per image, W WN / 8 groups (4 per wave); the 16-B chunk is XOR-swizzled by row
    const h16* asrc[NIMG][GA];
    const h16* wsrc[4];
#pragma unroll
    for (int i = 0; i < GA; ++i) {
        const int r = (i * NW + wave) * 8 + (lane >> 3);
        const int64_t gm = min(m0 + r, g.M - 1);
        asrc[0][i] = g.A + gm * g.lda + swz(r, lane & 7) * 8 + kbeg;
        if constexpr (LO) asrc[NIMG - 1][i] = g.A_lo + gm * g.lda + swz(r, lane & 7) * 8 + kbeg;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int r = (i * NW + wave) * 8 + (lane >> 3);
        wsrc[i] = g.W + (int64_t)min(n0 + r, g.N - 1) * g.ldw + swz(r, lane & 7) * 8 + kbeg;
    }
    auto stageA = [&](int slot, int k0) {
#pragma unroll
        for (int im = 0; im < NIMG; ++im)
#pragma unroll
            for (int i = 0; i < GA; ++i)
                __builtin_amdgcn_global_load_lds((const void*)(asrc[im][i] + k0),
                                                 (OSW_LDS void*)&la[(slot * NIMG + im) * WBM * BK + (i * NW + wave) * 8 * BK],
                                                 16, 0, 0);
    };
    auto stageW = [&](int slot, int k0) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            __builtin_amdgcn_global_load_lds((const void*)(wsrc[i] + k0),
                                             (OSW_LDS void*)&lw[slot * WN * BK + (i * NW + wave) * 8 * BK], 16, 0, 0);
    };
    f32x4 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nk = kc / BK;
    // issue order per thread: A(0) W(0) W(1) | per iteration kt: A(kt+1) W(kt+2)
    // (without LO, A(kt+2) rides with W(kt+2) as in the plain 3-slot ring)
    if constexpr (LO) {
        stageA(0, 0);
        stageW(0, 0);
        if (nk > 1) stageW(1, BK);
    } else {
        stageA(0, 0);
        stageW(0, 0);
        if (nk > 1) { stageA(1, BK); stageW(1, BK); }
    }
    for (int kt = 0; kt < nk; ++kt) {
        // tile kt has landed: younger than it are only tile kt+1's W (LO) or A+W
        if (kt + 1 < nk)
            wait_vmcnt<LO ? 4 : 4 + GA>();
        else
            wait_vmcnt<0>();
        __syncthreads();  // every thread's tile kt has landed; the slots refilled below are no longer read
        if constexpr (LO) {
            if (kt + 1 < nk) stageA((kt + 1) % ASL, (kt + 1) * BK);
            if (kt + 2 < nk) stageW((kt + 2) % WSL, (kt + 2) * BK);
        } else {
            if (kt + 2 < nk) { stageA((kt + 2) % WSL, (kt + 2) * BK); stageW((kt + 2) % WSL, (kt + 2) * BK); }
        }
        const int sa = kt % ASL;
        const h16* W = lw + (kt % WSL) * WN * BK;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int c = ks * 4 + (lane >> 4);
            h16x8 a[NIMG][4], b[2];
#pragma unroll
            for (int im = 0; im < NIMG; ++im)
#pragma unroll
                for (int mi = 0; mi < 4; ++mi) {
                    const int row = mi * 16 + (lane & 15);
                    a[im][mi] = *(const h16x8*)&la[(sa * NIMG + im) * WBM * BK + row * BK + swz(row, c) * 8];
                }
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) {
                const int row = wave * 32 + ni * 16 + (lane & 15);
                b[ni] = *(const h16x8*)&W[row * BK + swz(row, c) * 8];
            }
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int ni = 0; ni < 2; ++ni) {
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0][mi], b[ni], acc[mi][ni], 0, 0, 0);
                    if constexpr (LO)
                        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[NIMG - 1][mi], b[ni], acc[mi][ni], 0, 0, 0);
                }
        }
    }
    float* C = (float*)g.C + (g.kc > 0 ? (int64_t)blockIdx.z * g.M * g.ldc : 0);
    const float* bias = g.kc > 0 ? nullptr : g.bias;
    // the 64 x WN fp32 tile leaves through LDS (the W ring, free once every wave is past
    // its last K tile) as 8-B device-scope (write-through) stores, 512 B contiguous per
    // wave-instruction: the MFMA layout's 4-B stores scattered over 4 rows took ~half of
    // the beam logits GEMM (66 MB of fp32 at 320 rows).  Rows stay 8-B aligned for the
    // vocabulary's row stride (51866 floats), not 16-B.
    constexpr int TS = WN + 2;  // LDS row stride (floats) of the 64 x WN tile
    static_assert(WBM * TS * 4 <= WSL * WN * BK * 2, "the tile fits the W ring");
    float* T = (float*)lw;
    __syncthreads();
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = mi * 16 + (lane >> 4) * 4 + i;
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) {
                const int col = wave * 32 + ni * 16 + (lane & 15);
                const int n = min(n0 + col, g.N - 1);
                T[row * TS + col] = bias ? acc[mi][ni][i] + bias[n] : acc[mi][ni][i];
            }
        }
    __syncthreads();
#pragma unroll 4
    for (int f = threadIdx.x; f < WBM * WN / 2; f += NT) {
        const int row = f / (WN / 2), c2 = (f % (WN / 2)) * 2;
        const int m = m0 + row, n = n0 + c2;
        if (m >= g.M || n >= g.N) continue;
        float* dst = C + (int64_t)m * g.ldc + n;
        if (n + 1 < g.N) {
            const unsigned long long bits = (unsigned long long)__float_as_uint(T[row * TS + c2]) |
                                            ((unsigned long long)__float_as_uint(T[row * TS + c2 + 1]) << 32);
            __hip_atomic_store((unsigned long long*)dst, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(dst, T[row * TS + c2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <bool LO>
void launch_wide256(const GemmArgs& g, int ks, hipStream_t s) {
    constexpr int lds = wide_lds<256>(LO);
    set_lds_once((const void*)gemm_wide_kernel<LO, 256>, lds);
    gemm_wide_kernel<LO, 256><<<dim3((g.N + 255) / 256, (g.M + WBM - 1) / WBM, ks), 512, lds, s>>>(g);
}

void launch_wide(const GemmArgs& g, int ks, hipStream_t s) {
    // OSW_WIDE_N128=1 (A/B switch): the logits on the 64 x 128 tile too
    // OSW_WIDE256_ALL=1 (A/B switch): the split-K projections of beam rows on it as well
    static const bool n128 = getenv("OSW_WIDE_N128") != nullptr;
    static const bool all256 = getenv("OSW_WIDE256_ALL") != nullptr;
    if (!n128 && ((ks == 1 && g.kc == 0 && g.N >= 16384) || all256)) {
        if (g.A_lo) launch_wide256<true>(g, ks, s);
        else launch_wide256<false>(g, ks, s);
        return;
    }
    const dim3 grid((g.N + WBN - 1) / WBN, (g.M + WBM - 1) / WBM, ks);
    if (g.A_lo) gemm_wide_kernel<true><<<grid, 256, 0, s>>>(g);
    else gemm_wide_kernel<false><<<grid, 256, 0, s>>>(g);
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
        if (g.A_lo) gemm_skinny_kernel<MT, true, EPI, true><<<grid, 256, 0, s>>>(g, kc, part, ProArgs{});
        else gemm_skinny_kernel<MT, true, EPI, false><<<grid, 256, 0, s>>>(g, kc, part, ProArgs{});
    } else {
        if (g.A_lo) gemm_skinny_kernel<MT, false, EPI, true><<<grid, 256, 0, s>>>(g, kc, part, ProArgs{});
        else gemm_skinny_kernel<MT, false, EPI, false><<<grid, 256, 0, s>>>(g, kc, part, ProArgs{});
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

// split count: kc = 256 per workgroup (one register chunk of weights per wave)
// when that gives <= 2048 workgroups, else the smallest larger power-of-two
// multiple; K % 256 != 0 (small models) uses kc = 128.  Wide N (logits) runs
// unsplit and streams its K in 256-deep chunks.
int skinny_ksplit(int N, int K) {
    const int nbn = (N + 63) / 64;
    if (nbn >= 512) return 1;
    if (K % 256) return K / 128;
    // OSW_SKINNY_KC=k (A/B switch): K per workgroup at least k (fewer slabs, fewer workgroups)
    static const int kc_min = getenv("OSW_SKINNY_KC") ? atoi(getenv("OSW_SKINNY_KC")) : 256;
    if (kc_min > 256)
        for (int c = kc_min; c <= K; c += 128)
            if (K % c == 0 && c % 128 == 0) return K / c;
    int kc = 256;
    while ((K / kc) * nbn > 2048 && K % (2 * kc) == 0) kc *= 2;
    return K / kc;
}

// partial-slab mode: always writes part[ks][M][N] (no epilogue); returns ksplit.
// M > 64 (beam rows) runs ceil(M / 64) row groups on grid z; they read the same
// weights, so the weight stream comes from HBM once and from the MALL/L2 after.
// Hi/lo rows beyond 32 run as 32-row groups (MT = 2, 16 KiB of LDS): a 64-row workgroup
// (32 KiB) cannot start beside another lane's encoder GEMM tile, and the decoder then
// stalled for whole encoder tiles (51 us per projection instead of 16).
int launch_gemm_skinny_partial(const GemmArgs& g0, float* part, hipStream_t s) {
    static const bool no_pre = getenv("OSW_SKINNY_NOPRE") != nullptr;    // A/B switches
    static const bool no_pair = getenv("OSW_SKINNY_NOPAIR") != nullptr;
    GemmArgs g = g0;
    g.preload_w = no_pre ? 0 : 1;
    const int ks = skinny_ksplit(g.N, g.K);
    const int gr = (g.A_lo && g.M > 32) ? 32 : 64;
    const int nz = (g.M + gr - 1) / gr;
    g.pair_rows = (nz > 1 && !no_pair) ? 1 : 0;
    const int units = (g.N + 63) / 64 * ks;
    const dim3 grid = g.pair_rows ? dim3((unsigned)(8 * ((units + 7) / 8) * nz), 1, 1)
                                  : dim3((g.N + 63) / 64, ks, nz);
    const int kc = g.K / ks;
#define OSW_SKINNY_PART(MT_)                                                                     \
    do {                                                                                         \
        if (g.A_lo) gemm_skinny_kernel<MT_, false, EPI_F32, true><<<grid, 256, 0, s>>>(g, kc, part, ProArgs{}); \
        else gemm_skinny_kernel<MT_, false, EPI_F32, false><<<grid, 256, 0, s>>>(g, kc, part, ProArgs{}); \
    } while (0)
    switch (std::min(g.M, gr) <= 16 ? 1 : std::min(g.M, gr) <= 32 ? 2 : std::min(g.M, gr) <= 48 ? 3 : 4) {
        case 1: OSW_SKINNY_PART(1); break;
        case 2: OSW_SKINNY_PART(2); break;
        case 3: OSW_SKINNY_PART(3); break;
        default: OSW_SKINNY_PART(4); break;
    }
#undef OSW_SKINNY_PART
    return ks;
}

// launch_gemm_skinny_partial + the GELU tail (ProArgs::tail_*): fc1 of 9..64 decoder rows,
// whose reduce + bias + GELU then needs no kernel of its own.  Returns ksplit.
int launch_gemm_skinny_gelu_tail(const GemmArgs& g0, float* part, const ProArgs& pa, hipStream_t s) {
    static const bool no_pair = getenv("OSW_SKINNY_NOPAIR") != nullptr;
    GemmArgs g = g0;
    g.preload_w = 1;
    const int ks = skinny_ksplit(g.N, g.K);
    const int gr = (g.A_lo && g.M > 32) ? 32 : 64;
    const int nz = (g.M + gr - 1) / gr;
    g.pair_rows = (nz > 1 && !no_pair) ? 1 : 0;
    const int units = (g.N + 63) / 64 * ks;
    const dim3 grid = g.pair_rows ? dim3((unsigned)(8 * ((units + 7) / 8) * nz), 1, 1)
                                  : dim3((g.N + 63) / 64, ks, nz);
    const int kc = g.K / ks;
    if (!g.A_lo || g.M > 64 || g.N % 64)
        throw std::invalid_argument("GELU tail: hi/lo operand, <= 64 rows, N a multiple of 64");
    switch (std::min(g.M, gr) <= 16 ? 1 : 2) {
        case 1: gemm_skinny_kernel<1, false, EPI_F32, true, PRO_NONE, false, TAIL_GELU><<<grid, 256, 0, s>>>(g, kc, part, pa); break;
        default: gemm_skinny_kernel<2, false, EPI_F32, true, PRO_NONE, false, TAIL_GELU><<<grid, 256, 0, s>>>(g, kc, part, pa); break;
    }
    return ks;
}

// Mid-size M (beam-search decoder rows, 65..~640): the wide kernel's 64x128 tiles split
// over K so the grid still fills the chip; each split writes its own fp32 slab, reduced
// by the consumer kernel exactly like the skinny kernel's slabs.  Picks the largest
// split (K/ks a multiple of 64, >= 256 deep) that keeps the grid near 1024 workgroups
// (2 per CU).
// Fused small-batch form (<= PRO_ROWS hi/lo rows for PRO_RESLN, <= GELU_ROWS for PRO_GELU):
// the operand is built by the prologue (resln.h).  direct: one K range, EPI_F32 straight into g.C (the logits); otherwise the
// split-K slabs into part, as launch_gemm_skinny_partial.  Returns ksplit.
int launch_gemm_skinny_pro(const GemmArgs& g0, int pro, const ProArgs& pa, bool direct, float* part, hipStream_t s,
                           bool select, bool attn_tail) {
    GemmArgs g = g0;
    const int ks = direct ? 1 : skinny_ksplit(g.N, g.K);
    const dim3 grid((g.N + 63) / 64, ks, 1);
    const int kc = g.K / ks;
    static const bool wb_late = getenv("OSW_PRO_WB_LATE") != nullptr;  // A/B switch
    g.preload_w = wb_late ? 0 : 1;
    if (pro == PRO_GELU ? g.M > GELU_ROWS || kc > GELU_KC : g.M > PRO_ROWS)
        throw std::invalid_argument("fused GEMM prologue: rows or K range exceed its LDS image");
    if (select) {
        if (!direct || pro != PRO_RESLN || g.M != 1 || g.epi != EPI_F32 || g.ldc != g.N)
            throw std::invalid_argument("fused selection: batch-1 logits GEMM only");
        gemm_skinny_kernel<1, true, EPI_F32, true, PRO_RESLN, true><<<grid, 256, 0, s>>>(g, kc, part, pa);
        return ks;
    }
    if (attn_tail) {
        if (direct || pro != PRO_RESLN || g.M != 1 || g.N != 3 * pa.attn.H * 64 || !pa.tail_ticket)
            throw std::invalid_argument("attention tail: batch-1 qkv GEMM only");
        gemm_skinny_kernel<1, false, EPI_F32, true, PRO_RESLN, false, TAIL_ATTN><<<grid, 256, 0, s>>>(g, kc, part, pa);
        return ks;
    }
    if (direct) {
        if (pro == PRO_RESLN) gemm_skinny_kernel<1, true, EPI_F32, true, PRO_RESLN><<<grid, 256, 0, s>>>(g, kc, part, pa);
        else gemm_skinny_kernel<1, true, EPI_F32, true, PRO_GELU><<<grid, 256, 0, s>>>(g, kc, part, pa);
    } else {
        if (pro == PRO_RESLN) gemm_skinny_kernel<1, false, EPI_F32, true, PRO_RESLN><<<grid, 256, 0, s>>>(g, kc, part, pa);
        else gemm_skinny_kernel<1, false, EPI_F32, true, PRO_GELU><<<grid, 256, 0, s>>>(g, kc, part, pa);
    }
    return ks;
}

// one thread per 16-B piece of Wf: piece p = (blk * K/32 + st) * 64 + lane holds
// W[blk*16 + (lane & 15)][st*32 + 8 (lane >> 4) .. +8]
__global__ __launch_bounds__(256) void frag_pack_kernel(const h16* __restrict__ W, int64_t ldw, int N, int K,
                                                        h16* __restrict__ Wf, int64_t pieces) {
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= pieces) return;
    const int lane = (int)(p & 63);
    const int64_t t = p >> 6;
    const int ks = K >> 5;
    const int st = (int)(t % ks);
    const int n = (int)(t / ks) * 16 + (lane & 15);
    const int k = st * 32 + 8 * (lane >> 4);
    h16x8 v = {};
    if (n < N) v = *(const h16x8*)(W + (int64_t)n * ldw + k);
    *(h16x8*)(Wf + p * 8) = v;
}

void launch_frag_pack(const h16* W, int64_t ldw, int N, int K, h16* Wf, hipStream_t s) {
    const int64_t pieces = (int64_t)((N + 15) / 16) * (K / 32) * 64;
    frag_pack_kernel<<<(unsigned)((pieces + 255) / 256), 256, 0, s>>>(W, ldw, N, K, Wf, pieces);
}

int tiled_ksplit(int M, int N, int K) {
    const int tiles = ((M + WBM - 1) / WBM) * ((N + WBN - 1) / WBN);
    int best = 1;
    for (int ks = 1; ks <= K / BK; ++ks) {
        if (K % ks || (K / ks) % BK) continue;
        if ((K / ks) < 256 && ks > 1) break;
        if (tiles * ks > 1280) break;
        best = ks;
    }
    return best;
}

void launch_gemm_tiled_partial(const GemmArgs& g0, float* part, int ks, hipStream_t s) {
    GemmArgs g = g0;
    g.kc = g.K / ks;
    g.C = part;
    g.ldc = g.N;
    g.bias = nullptr;
    g.epi = EPI_F32;
    launch_wide(g, ks, s);
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

// every dynamic-LDS attribute of the GEMM kernels, set once (osw_create calls it)
void prepare_gemm_kernels() {
    static std::once_flag once;
    std::call_once(once, [] {
        constexpr int l256 = EPI_LDS > 2 * 2 * GB * BK * 2 ? EPI_LDS : 2 * 2 * GB * BK * 2;
        constexpr int l8p = EPI_LDS > 8 * HT * 2 ? EPI_LDS : 8 * HT * 2;
        auto each = [&](auto e) {
            constexpr int E = decltype(e)::value;
            set_lds_once((const void*)gemm256_kernel<E>, l256);
            set_lds_once((const void*)gemm8p_kernel<E, 0>, l8p);
            set_lds_once((const void*)gemm128_ring_kernel<E>, R128_LDS);
            set_lds_once((const void*)gemm8h_kernel<E, 0>, H8_LDS);
        };
        each(std::integral_constant<int, EPI_F16>{});
        each(std::integral_constant<int, EPI_F16_GELU>{});
        each(std::integral_constant<int, EPI_F32_RESID>{});
        each(std::integral_constant<int, EPI_F32_GELU_POS>{});
        each(std::integral_constant<int, EPI_F32>{});
        each(std::integral_constant<int, EPI_HEADS>{});
        set_lds_once((const void*)gemm8p_kernel<EPI_F32, 1>, l8p);
        set_lds_once((const void*)gemm8h_kernel<EPI_F32, 1>, H8_LDS);
        set_lds_once((const void*)gemm8p_kernel<EPI_F16, 2>, l8p);
        set_lds_once((const void*)gemm8p_kernel<EPI_F16_GELU, 2>, l8p);
        set_lds_once((const void*)gemm_wide_kernel<true, 256>, wide_lds<256>(true));
        set_lds_once((const void*)gemm_wide_kernel<false, 256>, wide_lds<256>(false));
    });
}

void launch_gemm_variant(const GemmArgs& g, int variant, hipStream_t s);

void launch_gemm(const GemmArgs& g, hipStream_t s) { launch_gemm_variant(g, 0, s); }

void launch_gemm_variant(const GemmArgs& g, int variant, hipStream_t s) {
    // few rows, very wide N, plain fp32 out (decoder logits): the 3-slot ring kernel; with
    // hi/lo activations (the decoder) at any row count
    static const bool no_wide = getenv("OSW_NO_WIDE") != nullptr;  // A/B switch
    const bool wide_ok = g.epi == EPI_F32 && g.kc == 0 && g.c_grp_rows == g.M && g.K % BK == 0 &&
                         (g.M <= WBM || g.A_lo);
    if (wide_ok && (variant == 5 || (variant == 0 && (g.A_lo || (g.N >= 16384 && !no_wide))))) {
        launch_wide(g, 1, s);
        return;
    }
    // Tile choice by tile count (every tile size gives identical results; measured on the
    // encoder shapes at 1-8 windows, tools/small_gemm_bench.py, profiles/r03_q_small_gemm.jsonl):
    // the 8-phase 256 tile from 180 tiles on (~0.7 of the CUs: at 2 windows fc1 47 vs 70 us
    // on the 128 tile, the cross-K/V GEMM at one window 48 vs 70 us), below that the 128
    // tile from 360 tiles, the 128 ring from 192, the 64 ring under it.
    static const int p8_min = [] {
        const char* e = getenv("OSW_8P_MIN");
        return e ? atoi(e) : 180;
    }();
    const int64_t big_tiles = (int64_t)((g.N + GB - 1) / GB) * ((g.M + GB - 1) / GB);
    if (variant == 0 && use_half_tile(g, big_tiles)) {
        switch (g.epi) {
            case EPI_F16: launch8h<EPI_F16>(g, s); return;
            case EPI_F16_GELU: launch8h<EPI_F16_GELU>(g, s); return;
            case EPI_F32_RESID: launch8h<EPI_F32_RESID>(g, s); return;
            case EPI_F32_GELU_POS: launch8h<EPI_F32_GELU_POS>(g, s); return;
            case EPI_F32: launch8h<EPI_F32>(g, s); return;
            default: launch8h<EPI_HEADS>(g, s); return;
        }
    }
    const bool big = !g.A_lo && (variant == 2 || (variant == 0 && big_tiles >= p8_min && g.N % 8 == 0 &&
                                                   !getenv("OSW_GEMM128")));

    static const bool two_phase = getenv("OSW_GEMM_2PHASE") != nullptr;  // A/B switch for the 8-phase schedule
    if (variant == 8) {  // debug: 8-phase, fp16 out / GELU fp16 out / no epilogue
        launch8p<EPI_F16>(g, s);
        return;
    }
    if (variant == 9) {
        launch8p<EPI_F32, 1>(g, s);
        return;
    }
    if (variant == 10) {
        launch8p<EPI_F16_GELU>(g, s);
        return;
    }
    if (variant == 14) {  // debug: the KW loop (W0 kept in registers), no epilogue / fp16 out
        launch8p<EPI_F32, 4>(g, s);
        return;
    }
    if (variant == 15) {
        launch8p<EPI_F16, 3>(g, s);
        return;
    }
    if (variant == 17) {  // debug: the half-width tile's main loop alone
        launch8h<EPI_F32, 1>(g, s);
        return;
    }
    if (variant == 18 || variant == 19) {  // debug: the half-width tile, fp16 / GELU fp16 out
        if (variant == 18) launch8h<EPI_F16>(g, s);
        else launch8h<EPI_F16_GELU>(g, s);
        return;
    }
    if (variant == 16 && !g.A_lo && g.N % 8 == 0) {  // the half-width 256 x 128 tile
        switch (g.epi) {
            case EPI_F16: launch8h<EPI_F16>(g, s); return;
            case EPI_F16_GELU: launch8h<EPI_F16_GELU>(g, s); return;
            case EPI_F32_RESID: launch8h<EPI_F32_RESID>(g, s); return;
            case EPI_F32_GELU_POS: launch8h<EPI_F32_GELU_POS>(g, s); return;
            case EPI_F32: launch8h<EPI_F32>(g, s); return;
            default: launch8h<EPI_HEADS>(g, s); return;
        }
    }
    if (variant == 12 || variant == 13) {  // debug: fp16 / GELU epilogues on accumulators not transposed
        if (variant == 12) launch8p<EPI_F16, 2>(g, s);
        else launch8p<EPI_F16_GELU, 2>(g, s);
        return;
    }
    if (variant == 4 || (variant == 0 && big && !two_phase)) {
        static const bool plain = [] {  // OSW_GEMM_TR=0: fp16 epilogues without transposed accumulators (A/B)
            const char* e = std::getenv("OSW_GEMM_TR");
            return e && e[0] == '0';
        }();
        switch (g.epi) {
            case EPI_F16: plain ? launch8p<EPI_F16, 2>(g, s) : launch8p<EPI_F16>(g, s); return;
            case EPI_F16_GELU: plain ? launch8p<EPI_F16_GELU, 2>(g, s) : launch8p<EPI_F16_GELU>(g, s); return;
            case EPI_F32_RESID: launch8p<EPI_F32_RESID>(g, s); return;
            case EPI_F32_GELU_POS: launch8p<EPI_F32_GELU_POS>(g, s); return;
            case EPI_F32: launch8p<EPI_F32>(g, s); return;
            default: launch8p<EPI_HEADS>(g, s); return;
        }
    }
    if (big) {
        switch (g.epi) {
            case EPI_F16: launch256<EPI_F16>(g, s); return;
            case EPI_F16_GELU: launch256<EPI_F16_GELU>(g, s); return;
            case EPI_F32_RESID: launch256<EPI_F32_RESID>(g, s); return;
            case EPI_F32_GELU_POS: launch256<EPI_F32_GELU_POS>(g, s); return;
            case EPI_F32: launch256<EPI_F32>(g, s); return;
            default: launch256<EPI_HEADS>(g, s); return;
        }
    }
    const int64_t tiles128 = (int64_t)((g.N + BN - 1) / BN) * ((g.M + BM - 1) / BM);
    // 128 ring for [r128_min, db128_min) tiles (OSW_RING128_MIN / OSW_DB128_MIN: A/B switches)
    static const int r128_min = [] {
        const char* e = getenv("OSW_RING128_MIN");
        return e ? atoi(e) : 192;
    }();
    static const int db128_min = [] {
        const char* e = getenv("OSW_DB128_MIN");
        return e ? atoi(e) : 360;
    }();
    // (16-B copy-out chunks: N and the row strides a multiple of 8)
    const bool r128_ok = g.N % 8 == 0 && (g.epi == EPI_HEADS || g.ldc % 8 == 0) && g.c_grp_stride % 8 == 0;
    if (r128_ok && (variant == 11 || (variant == 0 && g.kc == 0 && !g.A_lo && g.epi != EPI_F32 &&
                                      tiles128 >= r128_min && tiles128 < db128_min))) {
        switch (g.epi) {
            case EPI_F16: launch_ring128<EPI_F16>(g, s); return;
            case EPI_F16_GELU: launch_ring128<EPI_F16_GELU>(g, s); return;
            case EPI_F32_RESID: launch_ring128<EPI_F32_RESID>(g, s); return;
            case EPI_F32_GELU_POS: launch_ring128<EPI_F32_GELU_POS>(g, s); return;
            case EPI_F32: launch_ring128<EPI_F32>(g, s); return;
            default: launch_ring128<EPI_HEADS>(g, s); return;
        }
    }
    // fewer than 2 workgroups per CU on the 128 tile (small M: one or a few encoder
    // windows): the 64 tile, 4x the workgroups, identical results
    static const bool no_small = getenv("OSW_NO_TILE64") != nullptr;  // A/B switch
    if (variant == 6 || variant == 7 || (!no_small && variant == 0 && g.kc == 0 && tiles128 < r128_min)) {
        dim3 grid((g.N + 63) / 64, (g.M + 63) / 64);
        // the 4-slot ring (64 KB, 2 workgroups per CU): fc2 at one window 70 -> 39 us, the
        // out-projection 16 -> 14.5 us
        static const bool no_ring = getenv("OSW_NO_RING64") != nullptr;  // A/B switch
        if (variant == 6 || (variant == 0 && !no_ring)) {
            switch (g.epi) {
                case EPI_F16: gemm64_ring_kernel<EPI_F16><<<grid, NTHR, 0, s>>>(g); break;
                case EPI_F16_GELU: gemm64_ring_kernel<EPI_F16_GELU><<<grid, NTHR, 0, s>>>(g); break;
                case EPI_F32_RESID: gemm64_ring_kernel<EPI_F32_RESID><<<grid, NTHR, 0, s>>>(g); break;
                case EPI_F32_GELU_POS: gemm64_ring_kernel<EPI_F32_GELU_POS><<<grid, NTHR, 0, s>>>(g); break;
                case EPI_F32: gemm64_ring_kernel<EPI_F32><<<grid, NTHR, 0, s>>>(g); break;
                default: gemm64_ring_kernel<EPI_HEADS><<<grid, NTHR, 0, s>>>(g); break;
            }
            return;
        }
        switch (g.epi) {
            case EPI_F16: gemm_kernel<EPI_F16, 64><<<grid, NTHR, 0, s>>>(g); break;
            case EPI_F16_GELU: gemm_kernel<EPI_F16_GELU, 64><<<grid, NTHR, 0, s>>>(g); break;
            case EPI_F32_RESID: gemm_kernel<EPI_F32_RESID, 64><<<grid, NTHR, 0, s>>>(g); break;
            case EPI_F32_GELU_POS: gemm_kernel<EPI_F32_GELU_POS, 64><<<grid, NTHR, 0, s>>>(g); break;
            case EPI_F32: gemm_kernel<EPI_F32, 64><<<grid, NTHR, 0, s>>>(g); break;
            default: gemm_kernel<EPI_HEADS, 64><<<grid, NTHR, 0, s>>>(g); break;
        }
        return;
    }
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
