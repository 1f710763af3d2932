// Encoder self-attention (non-causal, T = 1500, head_dim 64) for gfx950.
//
// Flash-style: one workgroup = 4 waves = 128 queries of one (window, head); each
// wave owns 32 queries (two 16-query MFMA tiles).  K/V tiles of 64 keys are staged
// global -> LDS by 16-byte global_load_lds (double buffered; the 16-B chunk is
// XOR-swizzled through the source address as in gemm.hip).
//
//   Sᵀ = K · Qᵀ      v_mfma_f32_16x16x32_f16, A = K rows (ds_read_b128), B = Q (registers)
//                    -> each lane holds 16 scores of ONE query (lane & 15): the row
//                       max/sum need only 2 cross-lane xor-shuffles (16, 32)
//   Oᵀ += Vᵀ · Pᵀ    A = V read with ds_read_b64_tr_b16 (hardware transpose), B = P
//                    straight from the score registers (same k permutation on both
//                    operands), so O's query is again lane & 15 and the online-softmax
//                    rescale is lane-local.
// Softmax in fp32 base-2 with the 1/sqrt(64)·log2(e) scale folded into one multiply;
// P is rounded to fp16 for the PV MFMA (the oracle emulates exactly that).
//
// Layout in:  QKV head-major [3][nb][H][T][64] fp16 (written by the QKV GEMM epilogue)
// Layout out: O [nb*T][H*64] fp16 row-major (the out-projection GEMM's A operand)
#include "common.h"

#include <algorithm>
#include <cstdlib>

namespace osw {

namespace {
constexpr int QB = 128, KB = 64, HD = 64;

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }
// V's chunk swizzle.  A half-wave's ds_read_b64_tr_b16 reads 8 consecutive rows (an aligned
// 8-row group) x the two 16-B chunks {2dt, 2dt+1}; a 256-B bank row holds two 128-B rows, so
// the 4 even (odd) rows need pairwise different chunk pairs: c ^ (row & 6) gives them pair
// classes 0..3.  K's swizzle (row >> 1) gave rows 2n and 2n+2 the same pair: 2-way bank
// conflicts on every V read (SQ_LDS_BANK_CONFLICT = a third of the kernel's LDS cycles,
// profiles/r06_q_pmc_enc_1.txt).  Same bytes read, so identical results.
__device__ __forceinline__ int swzv(int row, int chunk) { return chunk ^ (row & 6); }

typedef __fp16 fp16x4_t __attribute__((__vector_size__(4 * sizeof(__fp16))));

__device__ __forceinline__ h16x4 ds_read_tr(const h16* p) {
    fp16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4f16((OSW_LDS fp16x4_t*)p);
    return __builtin_bit_cast(h16x4, v);
}

// LAZY: the running max is raised only when a tile's max exceeds it by more than 8 in
// the scaled base-2 domain (so every p = 2^(s*c - m) <= 2^8, exact in fp32 and in the
// fp16 P operand); O and l stay relative to the same stale max, so the normalised result
// is the same softmax, and the 32 O rescale multiplies per tile run only when some lane
// of the wave raised its max (rare after the first tiles) instead of every tile.
template <bool LAZY, int QT, bool PIPE>
__device__ __forceinline__ void enc_attn_unit(const h16* __restrict__ qkv, h16* __restrict__ out, int T, int H,
                                              int nb, int nqb, int nwg, int bid, h16 (&lds)[2][2][KB * HD]) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = lane >> 4, li = lane & 15;
    // XCD-aware order: the dispatcher deals workgroups round-robin over 8 XCDs; remap
    // (bijectively) so each XCD walks a contiguous run of (q-block, head, window)
    // indices with the q-block fastest -> one head's K/V stays in one XCD's L2.
    const int qq = nwg / 8, rr = nwg % 8, xcd = bid % 8;
    const int lin = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + bid / 8;
    const int qb = lin % nqb, h = (lin / nqb) % H, b = lin / (nqb * H);
    const int q0 = qb * (64 * QT) + wave * (16 * QT);
    const int64_t head_elems = (int64_t)T * HD;
    const h16* Qh = qkv + (((int64_t)0 * nb + b) * H + h) * head_elems;
    const h16* Kh = qkv + (((int64_t)1 * nb + b) * H + h) * head_elems;
    const h16* Vh = qkv + (((int64_t)2 * nb + b) * H + h) * head_elems;

    // Q fragments (B operand): lane: q = q0 + qt*16 + li, d = 32 s + 8 g + j
    h16x8 qf[QT][2];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        const int q = min(q0 + qt * 16 + li, T - 1);
#pragma unroll
        for (int s = 0; s < 2; ++s) qf[qt][s] = *(const h16x8*)(Qh + (int64_t)q * HD + 32 * s + 8 * g);
    }

    // glds pieces: 64 rows x 128 B = 8 KiB per tile = 8 wave-instructions; K: 2 per wave, V: 2 per wave
    auto stage_part = [&](int buf, int part, int k0) {
        const h16* src = part ? Vh : Kh;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int piece = i * 4 + wave;           // rows piece*8 .. +7
            const int r = piece * 8 + (lane >> 3);
            const int c = part ? swzv(r, lane & 7) : swz(r, lane & 7);
            const int key = min(k0 + r, T - 1);
            __builtin_amdgcn_global_load_lds((const void*)(src + (int64_t)key * HD + c * 8),
                                             (OSW_LDS void*)&lds[buf][part][piece * 8 * HD], 16, 0, 0);
        }
    };

    const float cs = 0.125f * 1.4426950408889634f;  // 1/sqrt(64) * log2(e)
    float mrun[QT], lrun[QT];
    f32x4 o[QT][4];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        mrun[qt] = -INFINITY;
        lrun[qt] = 0.f;
    }
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[qt][dt] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nkt = (T + KB - 1) / KB;

    // ---- Sᵀ = K Qᵀ : sc[qt][t] holds keys 16t + 4g + i for query li
    auto qk = [&](const h16* Kl, f32x4 (&sc)[QT][4]) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int row = 16 * t + li;
            const h16x8 k0f = *(const h16x8*)&Kl[row * HD + swz(row, g) * 8];
            const h16x8 k1f = *(const h16x8*)&Kl[row * HD + swz(row, 4 + g) * 8];
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(k0f, qf[qt][0], a, 0, 0, 0);
                a = __builtin_amdgcn_mfma_f32_16x16x32_f16(k1f, qf[qt][1], a, 0, 0, 0);
                sc[qt][t] = a;
            }
        }
    };
    // ---- online softmax of tile kt's scores, then Oᵀ += Vᵀ Pᵀ.  TAIL: the last tile,
    // whose keys past T are masked (a separate instantiation: the masking selects cost ~50
    // VALU ops per tile in every tile when the condition was a runtime flag, in a VALU-bound
    // loop)
    auto softmax_pv = [&](int kt, auto tail_c, f32x4 (&sc)[QT][4], const h16* Vl) {
        constexpr bool tail = decltype(tail_c)::value;
        const int k0 = kt * KB;
        // (lane-local per query; 4 lanes g=0..3 share a query).  VALU is this loop's bound
        // at d = 64 (≈ 2x the MFMA cycles), so: the running max is kept on raw scores and
        // the 1/sqrt(d)*log2(e) scale folds into one FMA per score, keys past T are masked
        // only in the last tile, and exp2 is the bare v_exp_f32 (results below 2^-126 flush
        // to 0, irrelevant next to the row maximum's 1).
        h16x8 pf[QT][2];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            float mx = -INFINITY;
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    if constexpr (tail)
                        if (k0 + 16 * t + 4 * g + i >= T) sc[qt][t][i] = -INFINITY;
                    mx = fmaxf(mx, sc[qt][t][i]);
                }
            mx = fmaxf(mx, xor_lane<16>(mx));
            mx = fmaxf(mx, xor_lane<32>(mx));
            float mnew = fmaxf(mrun[qt], mx);
            bool rescale = true;
            if constexpr (LAZY) {
                // keep the stale max while the tile stays within 2^8 of it (the first tile
                // always takes its max: mrun starts at -inf)
                if ((mnew - mrun[qt]) * cs <= 8.0f) mnew = mrun[qt];
                rescale = __any(mnew != mrun[qt]);
            }
            const float alpha = __builtin_amdgcn_exp2f((mrun[qt] - mnew) * cs);
            mrun[qt] = mnew;
            const float mcs = -mnew * cs;
            float ls = 0.f;
            float p[4][4];
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    p[t][i] = __builtin_amdgcn_exp2f(fmaf(sc[qt][t][i], cs, mcs));
                    ls += p[t][i];
                }
            lrun[qt] = lrun[qt] * alpha + ls;
            if (rescale) {
#pragma unroll
                for (int dt = 0; dt < 4; ++dt) o[qt][dt] *= alpha;
            }
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                h16x8 f;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    f[j] = (h16)p[2 * s][j];
                    f[4 + j] = (h16)p[2 * s + 1][j];
                }
                pf[qt][s] = f;
            }
        }
        // ---- Oᵀ += Vᵀ Pᵀ ; A = V via transposed LDS reads
#pragma unroll
        for (int s = 0; s < 2; ++s) {
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                const int q4 = li >> 2, p4 = li & 3;
                const int col = 16 * dt + 4 * p4;
                const int ch = col >> 3, within = col & 7;
                const int r0 = 32 * s + 4 * g + q4;
                const int r1 = r0 + 16;
                const h16x4 va = ds_read_tr(&Vl[r0 * HD + swzv(r0, ch) * 8 + within]);
                const h16x4 vb = ds_read_tr(&Vl[r1 * HD + swzv(r1, ch) * 8 + within]);
                h16x8 vf;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    vf[j] = va[j];
                    vf[4 + j] = vb[j];
                }
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
                    o[qt][dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf, pf[qt][s], o[qt][dt], 0, 0, 0);
            }
        }
    };
    const bool last_partial = nkt * KB > T;
    if constexpr (!PIPE) {
        // one K/V tile per step, the next tile's K and V staged at its start
        stage_part(0, 0, 0);
        stage_part(0, 1, 0);
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        auto tile = [&](int kt, auto tail_c) {
            const int buf = kt & 1;
            if (kt + 1 < nkt) {
                stage_part(buf ^ 1, 0, (kt + 1) * KB);
                stage_part(buf ^ 1, 1, (kt + 1) * KB);
            }
            f32x4 sc[QT][4];
            qk(lds[buf][0], sc);
            softmax_pv(kt, tail_c, sc, lds[buf][1]);
            __builtin_amdgcn_s_waitcnt(0);
            __syncthreads();
        };
        for (int kt = 0; kt < nkt - (last_partial ? 1 : 0); ++kt) tile(kt, std::false_type{});
        if (last_partial) tile(nkt - 1, std::true_type{});
    } else {
        // Software-pipelined (PIPE): step kt computes tile kt+1's scores (MFMA) in the same
        // block as tile kt's softmax (VALU) and PV (MFMA), so one wave's matrix and vector
        // work interleave instead of taking turns.  K(j) lives in lds[j & 1][0] and V(j) in
        // lds[j & 1][1]; step kt stages K(kt+2) into the K half its own scores came from and
        // V(kt+1) into the V half tile kt-1's PV read, both free after the previous step's
        // barrier, and reads K(kt+1) and V(kt), both landed before it.  The same MFMAs and
        // softmax per tile in the same order as the unpipelined form: identical results.
        stage_part(0, 0, 0);
        stage_part(0, 1, 0);
        if (nkt > 1) stage_part(1, 0, KB);
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        f32x4 sa[QT][4], sb[QT][4];
        qk(lds[0][0], sa);
        auto step = [&](int kt, auto tail_c, auto next_c, f32x4 (&cur)[QT][4], f32x4 (&nxt)[QT][4]) {
            constexpr bool next = decltype(next_c)::value;
            const int buf = kt & 1;
            if (kt + 2 < nkt) stage_part(buf, 0, (kt + 2) * KB);
            if (kt + 1 < nkt) stage_part(buf ^ 1, 1, (kt + 1) * KB);
            if constexpr (next) qk(lds[buf ^ 1][0], nxt);
            softmax_pv(kt, tail_c, cur, lds[buf][1]);
            __builtin_amdgcn_s_waitcnt(0);
            __syncthreads();
        };
        // steps 0 .. nkt-2 have a next tile; the roles of sa / sb alternate (unrolled by 2,
        // so no register copies)
        int kt = 0;
        for (; kt + 1 < nkt - 1; kt += 2) {
            step(kt, std::false_type{}, std::true_type{}, sa, sb);
            step(kt + 1, std::false_type{}, std::true_type{}, sb, sa);
        }
        if (kt < nkt - 1) {
            step(kt, std::false_type{}, std::true_type{}, sa, sb);
            ++kt;
            if (last_partial) step(kt, std::true_type{}, std::false_type{}, sb, sa);
            else step(kt, std::false_type{}, std::false_type{}, sb, sa);
        } else {
            if (last_partial) step(kt, std::true_type{}, std::false_type{}, sa, sb);
            else step(kt, std::false_type{}, std::false_type{}, sa, sb);
        }
    }

    // ---- normalise and store: lane holds O[q = li][d = 16 dt + 4 g + i]
    const int D = H * HD;
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        float l = lrun[qt];
        l += xor_lane<16>(l);
        l += xor_lane<32>(l);
        const float inv = 1.0f / l;
        const int q = q0 + qt * 16 + li;
        if (q >= T) continue;
        h16* orow = out + ((int64_t)b * T + q) * D + h * HD;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            h16x4 v;
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = (h16)(o[qt][dt][i] * inv);
            *(h16x4*)(orow + 16 * dt + 4 * g) = v;
        }
    }
}

// Persistent over the (q-block, head, window) units when the grid is capped (workgroup b
// runs units b, b + grid, ...; grid a multiple of 8, so a unit keeps its XCD): like the
// encoder GEMM, the attention then leaves a quarter of the CUs to another lane's decoder.
// QT: 16-query MFMA tiles per wave (2: 128 queries per workgroup; 1: 64, for one or two
// windows, where 128-query blocks leave CUs idle: 240 workgroups at one window).  A
// query's arithmetic does not depend on the queries beside it (the lazy max is per lane;
// a skipped rescale is a multiply by exactly 1), so both forms give identical results.
template <bool LAZY, int QT, bool PIPE>
__global__ __launch_bounds__(256, 2) void enc_attn_kernel(const h16* __restrict__ qkv, h16* __restrict__ out,
                                                          int T, int H, int nb, int nqb) {
    __shared__ __attribute__((aligned(16))) h16 lds[2][2][KB * HD];  // [buf][K|V] 32 KiB
    const int nwg = nqb * H * nb;
    for (int vb = blockIdx.x; vb < nwg; vb += gridDim.x) {
        enc_attn_unit<LAZY, QT, PIPE>(qkv, out, T, H, nb, nqb, nwg, vb, lds);
        __syncthreads();  // the LDS ring is the next unit's
    }
}
}  // namespace

void launch_enc_attn(const h16* qkv, h16* out, int T, int H, int nb, hipStream_t s) {
    // 64-query blocks while 128-query ones would give < 2 workgroups per CU (OSW_ATTN_QB: force 64 / 128)
    static const int qb_env = [] {
        const char* e = std::getenv("OSW_ATTN_QB");
        return e ? atoi(e) : 0;
    }();
    const bool small = qb_env ? qb_env == 64 : (int64_t)((T + QB - 1) / QB) * H * nb < 512;
    const int nqb = small ? (T + 63) / 64 : (T + QB - 1) / QB;
    const int nwg = nqb * H * nb;
    static const bool eager = [] {  // OSW_ATTN_LAZY=0: rescale O on every tile (A/B)
        const char* e = std::getenv("OSW_ATTN_LAZY");
        return e && e[0] == '0';
    }();
    // optional grid cap (OSW_ATTN_GRID, A/B only): a capped grid loops over the units.  Default
    // one workgroup per unit: capping at 2 WGs/CU on 3/4 of the CUs (as the GEMM) measured
    // 4843/4814 vs 4858/4853 audio-s/s uncapped, 256 and 512 both ~4810 (profiles r03_i).
    static const int cap = [] {
        if (const char* e = std::getenv("OSW_ATTN_GRID")) return std::max(8, atoi(e) / 8 * 8);
        return 1 << 30;
    }();
    const int grid = std::min(nwg, cap);
    static const bool pipe = [] {  // OSW_ATTN_PIPE=1: the software-pipelined step (A/B)
        const char* e = std::getenv("OSW_ATTN_PIPE");
        return e && e[0] == '1';
    }();
#define OSW_ATTN_LAUNCH(L, Q, P) enc_attn_kernel<L, Q, P><<<grid, 256, 0, s>>>(qkv, out, T, H, nb, nqb)
    if (small) {
        if (eager) pipe ? OSW_ATTN_LAUNCH(false, 1, true) : OSW_ATTN_LAUNCH(false, 1, false);
        else pipe ? OSW_ATTN_LAUNCH(true, 1, true) : OSW_ATTN_LAUNCH(true, 1, false);
    } else {
        if (eager) pipe ? OSW_ATTN_LAUNCH(false, 2, true) : OSW_ATTN_LAUNCH(false, 2, false);
        else pipe ? OSW_ATTN_LAUNCH(true, 2, true) : OSW_ATTN_LAUNCH(true, 2, false);
    }
#undef OSW_ATTN_LAUNCH
}

}  // namespace osw
