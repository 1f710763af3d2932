// Cross-attention over the encoder output E itself ("E-form") for greedy decoder batches
// of >= EX_MIN_ROWS windows (osw.hip decoder_step).
//
// Whisper's cross-attention keys and values are linear in E (k_proj has no bias):
//   K_h = E·Wk_hᵀ,  V_h = E·Wv_hᵀ + bv_h     (E: [1500][D] per window, Wk_h/Wv_h: [64][D])
// so for a query q_h
//   softmax(q_h·K_hᵀ/8)·V_h = (Σ_t p_t E_t / Σ_t p_t)·Wv_hᵀ + bv_h,   p_t = exp(q'_h·E_t - m),
//   q'_h = Wk_hᵀ q_h / 8   (D values per head instead of 64).
// The cached-K/V form reads K and V of all heads, 2 x 1500 x D fp16 per window and layer;
// this form reads E ONCE for all heads: 1500 x D.  The bytes per decoded token halve
// (30.72 -> 15.36 MB per window at large-v3-turbo) for 20x the MFMA work (still far
// below the HBM time), and the result skips the fp16 rounding of K and V.
//
// Per layer: ex_qk (q' of every head: the q projection's split-K slabs reduced as
// dec_xattn_chunk_kernel reduces them, then x Wk_h on MFMA), exattn (per (window, key
// chunk): scores of all heads, online softmax, P·E, fp32 partials), ex_merge (the 4 chunk
// partials of a (window, head) in fixed order, normalised, as an hi/lo fp16 pair), then the
// V projection (gemm_skinny_kernel with a per-head A offset) and its split-K reduce
// (+ bv) into the out-projection's operand.  Every window's arithmetic is independent of
// the batch, and the chunk merge order is fixed.
//
// exattn layout: 64 x NW threads; wave w owns the E columns [w*JW, (w+1)*JW) for both the
// scores (its partial dot products are summed over the waves in LDS, in wave order) and
// P·E (its O columns).  Each wave stages only its own column slice of each 16-key E tile
// (3-slot LDS ring, two tiles in flight), so E staging needs no barrier; one barrier per
// tile hands the partial scores over.
//   Sᵀ = E_tile · q'ᵀ   v_mfma_f32_16x16x32_f16: A = E rows (ds_read_b128), B = q' (hi, lo)
//                       -> lane holds keys 4g + i of head li (g = lane >> 4, li = lane & 15)
//   Oᵀ += E_tileᵀ · Pᵀ  v_mfma_f32_16x16x16_f16: A = E columns (ds_read_b64_tr_b16), B = P
//                       (hi, lo) straight from the softmax registers
#include "decode.h"
#include "ldsasm.h"

#include <cstdlib>

namespace osw {

namespace {
constexpr int EX_KT = 16;    // keys per tile
constexpr int EX_NBUF = 3;   // E tile ring slots per wave

__device__ __forceinline__ int ex_swz(int r) { return 2 * ((r >> 2) & 1) + ((r >> 3) & 1); }

// q' of a window in the scores' B-fragment order: k32 step j / 32, head tile h / 16, lane
// 16 ((j % 32) / 8) + h % 16, element j % 8 -- one wave's fragment is 1 KiB contiguous
__device__ __forceinline__ int ex_qfrag(int h, int j) {
    return (((j >> 5) * 2 + (h >> 4)) * 64 + 16 * ((j & 31) >> 3) + (h & 15)) * 8 + (j & 7);
}


// q' = (Wk_h^T q16_h) / 8 for every row and head; grid (H, D / 128), 256 threads.
// q16 = fp16(bias + Σ_k part[k]) (slabs summed in order; the rounding point the oracle's
// "dec_q" emulates).  kT: Wk of this layer as [H][D][64] (kT[h][j][dd] = Wk[h*64 + dd][j]).
// Rows past `rows` of the q image are zero.
__global__ __launch_bounds__(256) void ex_qk_kernel(const float* __restrict__ part, int ks, int64_t slab,
                                                    const float* __restrict__ bias, int rows, int D,
                                                    const h16* __restrict__ kT, h16* __restrict__ qp,
                                                    int64_t qlo) {
    constexpr int MAXR = 128;
    __shared__ __attribute__((aligned(16))) h16 qs[MAXR][64 + 8];
    const int h = blockIdx.x, j0 = blockIdx.y * 128;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, g = lane >> 4, li = lane & 15;
    const int mt_n = (rows + 15) / 16;
    // this wave's Wk columns first: their latency overlaps the slab reduction
    const h16* kh = kT + (int64_t)h * D * 64;
    h16x8 b[2][2];
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        const int j = j0 + (2 * wv + n) * 16 + li;
        b[n][0] = *(const h16x8*)(kh + (int64_t)j * 64 + 8 * g);
        b[n][1] = *(const h16x8*)(kh + (int64_t)j * 64 + 32 + 8 * g);
    }
    // q rows of this head, 4 columns per thread and pass; the slab loads of a pass are
    // independent, summed in slab order
    const float4 bb = *(const float4*)(bias + h * 64 + 4 * (tid & 15));
    for (int r0 = tid >> 4; r0 < mt_n * 16; r0 += 64) {
        float4 v[4];
        int nr = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int r = r0 + 16 * u;
            v[u] = float4{0.f, 0.f, 0.f, 0.f};
            if (r < mt_n * 16) nr = u + 1;
        }
        for (int s = 0; s < ks; ++s) {
            float4 x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int r = r0 + 16 * u;
                x[u] = (u < nr && r < rows) ? *(const float4*)(part + s * slab + (int64_t)r * D + h * 64 + 4 * (tid & 15))
                                            : float4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] += x[u];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int r = r0 + 16 * u;
            if (u >= nr) break;
            const bool in = r < rows;
            h16* q = &qs[r][4 * (tid & 15)];
            q[0] = (h16)(in ? bb.x + v[u].x : 0.f);
            q[1] = (h16)(in ? bb.y + v[u].y : 0.f);
            q[2] = (h16)(in ? bb.z + v[u].z : 0.f);
            q[3] = (h16)(in ? bb.w + v[u].w : 0.f);
        }
    }
    __syncthreads();
    // MFMA: C[r][j] = Σ_dd qs[r][dd] kT[h][j][dd]; wave: n-tiles 2 wv, 2 wv + 1 (16 j each)
#pragma unroll
    for (int n = 0; n < 2; ++n) {
        const int j = j0 + (2 * wv + n) * 16 + li;
        for (int mt = 0; mt < mt_n; ++mt) {
            const int r = mt * 16 + li;
            const h16x8 a0 = *(const h16x8*)&qs[r][8 * g];
            const h16x8 a1 = *(const h16x8*)&qs[r][32 + 8 * g];
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b[n][0], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b[n][1], acc, 0, 0, 0);
            // D[row = 4g + i][col = li]: row mt*16 + 4g + i, column j
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = mt * 16 + 4 * g + i;
                if (row >= rows) continue;
                const float v = acc[i] * 0.125f;  // 1/sqrt(64), exact
                const h16 hi = (h16)v;
                const int64_t o = (int64_t)row * EX_HP * D + ex_qfrag(h, j);
                qp[o] = hi;
                qp[o + qlo] = (h16)(v - (float)hi);
            }
        }
    }
}

// One (window, key chunk): partial (m, l, O[D]) per head over the chunk's keys.
// Per 16-key tile, software-pipelined so that one stretch of MFMA work holds the scores of
// tile t+1 AND P·E of tile t:
//   [P(t), alpha(t) from LDS; rescale O]  scores(t+1) -> Sp  P·E(t)  restage  | barrier |
//   softmax(t+1): lane = (head, key), partials summed in wave order -> P(t+1), alpha(t+1)  | barrier |
// The softmax of a head lives in one wave (its 16 keys on 16 lanes), so the running max and
// sum are that wave's registers; every wave reads P as the B operand of
// v_mfma_f32_32x32x16_f16 (N = the 32 padded heads, K = the tile's 16 keys).
template <int NW, int JW>
__global__ __launch_bounds__(NW * 64, 1) void exattn_kernel(const h16* __restrict__ E, const h16* __restrict__ qp,
                                                            int64_t qlo, int W, int T, int H,
                                                            float* __restrict__ ws, int pstride,
                                                            const SelState* __restrict__ st) {
    constexpr int D = NW * JW, NS = JW / 32, NM = JW / 32, CH = JW / 8, NI = JW / 32;
    constexpr int EPL = (EX_HP * EX_KT) / (NW * 64);  // softmax entries per lane
    static_assert(JW % 32 == 0, "a wave's column slice is whole k32 steps and 32-column M tiles");
    static_assert(EPL * NW * 64 == EX_HP * EX_KT, "softmax entries spread evenly over the lanes");
    __shared__ __attribute__((aligned(16))) h16 Es[NW][EX_NBUF][EX_KT * JW];  // per wave: its ring slots
    __shared__ __attribute__((aligned(16))) f32x4 Sp[NW][2][64];      // partial scores, MFMA C layout
    __shared__ __attribute__((aligned(16))) h16 Pt[2][EX_HP][EX_KT];  // P hi, lo as [head][key]
    __shared__ float Al[EX_HP];                                        // rescale factor per head
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, g = lane >> 4, li = lane & 15;
    // blocks b, b + 8, b + 16, .. (one XCD: b % 8) hold the chunks of one window, so its q'
    // comes from HBM once and from that XCD's L2 for the other chunks
    const int x = blockIdx.x % (8 * EX_CHUNKS);
    const int w = 8 * (blockIdx.x / (8 * EX_CHUNKS)) + x % 8, c = x / 8;
    if (w >= W) return;
    if (st[w].done) return;  // a finished window: its outputs are never used
    const int per = (T + EX_CHUNKS - 1) / EX_CHUNKS;
    const int k0 = c * per, nk = min(T, k0 + per) - k0;
    const int ntiles = (nk + EX_KT - 1) / EX_KT;

    // q' B fragments: B[k = j][col = head] = q'[head = ht*16 + li][wv*JW + 32 s + 8 g + i]
    h16x8 qh[NS][2], ql[NS][2];
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int ht = 0; ht < 2; ++ht) {
            const h16* p = qp + (int64_t)w * EX_HP * D + ex_qfrag(ht * 16 + li, wv * JW + 32 * s + 8 * g);
            const bool real = ht * 16 + li < H;  // padded heads: q' = 0, not loaded
            qh[s][ht] = real ? *(const h16x8*)p : h16x8{};
            ql[s][ht] = real ? *(const h16x8*)(p + qlo) : h16x8{};
        }
    // this wave's slice of a 16-key tile: LDS position (row r, chunk cs) holds E chunk cs ^ swz(r).
    // Buffer loads: a 32-bit per-lane offset from the chunk's (block-uniform) base, the wave's
    // column offset in soffset, so the stage addresses cost few VGPRs
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(E + ((int64_t)w * T + k0) * D), (short)0, nk * D * 2, 0x00020000);
    const int wcol = __builtin_amdgcn_readfirstlane(wv * JW * 2);
    auto stage = [&](int buf, int t) {
        const int kb = t * EX_KT;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int slot = i * 64 + lane, r = slot / CH, cs = slot % CH;
            const int key = min(kb + r, nk - 1);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (OSW_LDS void*)&Es[wv][buf][i * 64 * 8], 16,
                                                     key * (D * 2) + 16 * (cs ^ ex_swz(r)), wcol, 0, 0);
        }
    };
    stage(0, 0);
    if (ntiles > 1) stage(1, 1);
    if (ntiles > 2) stage(2, 2);
    // the q' fragments are used by every tile: have the compiler's wait for them here (it
    // counts the E tiles issued after them), not at their first use inside the tile loop,
    // where it becomes a vmcnt(0) on every tile
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int ht = 0; ht < 2; ++ht) {
            asm_landed(qh[s][ht]);
            asm_landed(ql[s][ht]);
        }

    // a landed tile into registers: E rows (the scores' A operand) and E columns by
    // transposed reads (P·E's A operand: lane (j = lane & 31, keys 8 (lane >> 5) .. + 7) of
    // each 32-column M tile; 16-lane group g reads keys 8 (g >> 1) + 4 r + (li >> 2), columns
    // 16 (g & 1) + 4 (li & 3) .. + 3 of the tile).  The slot is free again once the reads
    // have returned, so it is restaged right away: the ring keeps 3 tiles in flight.
    const int trq = li >> 2, trp = li & 3;
    auto read_tile = [&](int t, h16x8 (&arow)[NS], h16x8 (&acol)[NM]) {
        const h16* El = Es[wv][t % EX_NBUF];
#pragma unroll
        for (int s = 0; s < NS; ++s) arow[s] = asm_read_b128(&El[li * JW + 8 * ((4 * s + g) ^ ex_swz(li))]);
        h16x4 tr[NM][2];
#pragma unroll
        for (int m = 0; m < NM; ++m)
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const int row = 8 * (g >> 1) + 4 * r + trq, lc = 4 * m + 2 * (g & 1) + (trp >> 1);
                tr[m][r] = asm_read_tr(&El[row * JW + 8 * (lc ^ ex_swz(row)) + 4 * (trp & 1)]);
            }
        asm_wait_lgkm();
#pragma unroll
        for (int s = 0; s < NS; ++s) asm_landed(arow[s]);
#pragma unroll
        for (int m = 0; m < NM; ++m) {
            asm_landed(tr[m][0]);
            asm_landed(tr[m][1]);
            acol[m] = __builtin_shufflevector(tr[m][0], tr[m][1], 0, 1, 2, 3, 4, 5, 6, 7);
        }
        if (t + EX_NBUF < ntiles) stage(t % EX_NBUF, t + EX_NBUF);
    };
    // partial scores of a tile over this wave's columns -> Sp[wv]
    auto scores = [&](const h16x8 (&arow)[NS]) {
        f32x4 sp[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int ht = 0; ht < 2; ++ht) {
                sp[ht] = __builtin_amdgcn_mfma_f32_16x16x32_f16(arow[s], qh[s][ht], sp[ht], 0, 0, 0);
                sp[ht] = __builtin_amdgcn_mfma_f32_16x16x32_f16(arow[s], ql[s][ht], sp[ht], 0, 0, 0);
            }
        Sp[wv][0][lane] = sp[0];
        Sp[wv][1][lane] = sp[1];
    };
    // softmax of tile t: lane entry e is (head, key) = ((wv * EPL + e) * 64 + lane) / 16, % 16
    const float cs2 = 1.4426950408889634f;  // log2(e): the 1/sqrt(64) is in q'
    float mrun[EPL], lrun[EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
        mrun[e] = -INFINITY;
        lrun[e] = 0.f;
    }
    auto softmax = [&](int t) {
#pragma unroll
        for (int e = 0; e < EPL; ++e) {
            const int id = (wv * EPL + e) * 64 + lane, head = id >> 4, key = id & 15;
            const float* sp = (const float*)&Sp[0][head >> 4][16 * (key >> 2) + (head & 15)] + (key & 3);
            float part[NW];
#pragma unroll
            for (int u = 0; u < NW; ++u) part[u] = asm_read_f32(sp + u * 2 * 64 * 4);
            asm_wait_lgkm();
#pragma unroll
            for (int u = 0; u < NW; ++u) asm_landed(part[u]);
            float s = part[0];
#pragma unroll
            for (int u = 1; u < NW; ++u) s += part[u];
            if (t * EX_KT + key >= nk) s = -INFINITY;  // keys past the chunk
            float mx = fmaxf(s, xor_lane<1>(s));
            mx = fmaxf(mx, xor_lane<2>(mx));
            mx = fmaxf(mx, xor_lane<4>(mx));
            mx = fmaxf(mx, xor_lane<8>(mx));
            // lazy running max (as enc_attn): raised only when the tile exceeds it by 2^8
            float mnew = fmaxf(mrun[e], mx);
            if ((mnew - mrun[e]) * cs2 <= 8.0f) mnew = mrun[e];
            const float alpha = __builtin_amdgcn_exp2f((mrun[e] - mnew) * cs2);
            mrun[e] = mnew;
            const float p = __builtin_amdgcn_exp2f(fmaf(s, cs2, -mnew * cs2));
            lrun[e] = fmaf(lrun[e], alpha, p);
            const h16 hi = (h16)p;
            Pt[0][head][key] = hi;
            Pt[1][head][key] = (h16)(p - (float)hi);
            if (key == 0) Al[head] = alpha;
        }
    };

    f32x16 o[NM];
#pragma unroll
    for (int m = 0; m < NM; ++m)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[m][i] = 0.f;

    // tile k+3 is issued once tile k is in registers; waiting for tile k leaves tiles k+1
    // and k+2 in flight
    auto wait_tile = [&](int k) {
        const int after = min(ntiles - 1 - k, 2);
        after == 2 ? asm_wait_vmcnt<2 * NI>() : after == 1 ? asm_wait_vmcnt<NI>() : asm_wait_vmcnt<0>();
    };
    h16x8 arow[NS], acol[NM];
    wait_tile(0);
    read_tile(0, arow, acol);
    scores(arow);
    asm_lds_barrier();
    softmax(0);
    asm_lds_barrier();
    for (int t = 0; t < ntiles; ++t) {
        // (LDS reads as asm throughout the loop: ldsasm.h)
        h16x8 bh = asm_read_b128(&Pt[0][lane & 31][8 * (lane >> 5)]);
        h16x8 bl = asm_read_b128(&Pt[1][lane & 31][8 * (lane >> 5)]);
        float alpha = asm_read_f32(&Al[lane & 31]);
        asm_wait_lgkm();
        asm_landed(bh);
        asm_landed(bl);
        asm_landed(alpha);
        if (__any(alpha != 1.0f)) {
#pragma unroll
            for (int m = 0; m < NM; ++m) o[m] *= alpha;
        }
#pragma unroll
        for (int m = 0; m < NM; ++m) {
            o[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(acol[m], bh, o[m], 0, 0, 0);
            o[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(acol[m], bl, o[m], 0, 0, 0);
        }
        if (t + 1 < ntiles) {
            wait_tile(t + 1);
            read_tile(t + 1, arow, acol);
            scores(arow);
            asm_lds_barrier();
            softmax(t + 1);
            asm_lds_barrier();
        }
    }
    // ---- partials: ws[w][c][head] = {m, l, pad x 6, O[D]} (plain stores: ex_merge is the next launch)
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
        const int id = (wv * EPL + e) * 64 + lane, head = id >> 4, key = id & 15;
        float l = lrun[e];
        l += xor_lane<1>(l);
        l += xor_lane<2>(l);
        l += xor_lane<4>(l);
        l += xor_lane<8>(l);
        if (key == 0 && head < H) {
            float* dst = ws + (((int64_t)w * EX_CHUNKS + c) * H + head) * pstride;
            dst[0] = mrun[e];
            dst[1] = l;
        }
    }
    // O through this wave's own ring slots (no barrier: nothing else reads or fills them any
    // more) so each head's JW columns leave as whole 16-byte runs of one row
    constexpr int OS = JW + 4;  // row stride in floats: the 16 heads of a write on distinct banks
    static_assert((D / 64) * OS * 4 <= EX_NBUF * EX_KT * JW * 2, "O of every head fits the wave's slots");
    float* Ol = (float*)&Es[wv][0][0];
    const int head = lane & 31;
    if (head < H) {
#pragma unroll
        for (int m = 0; m < NM; ++m)
#pragma unroll
            for (int b = 0; b < 4; ++b)
                *(f32x4*)&Ol[head * OS + 32 * m + 8 * b + 4 * (lane >> 5)] =
                    f32x4{o[m][4 * b], o[m][4 * b + 1], o[m][4 * b + 2], o[m][4 * b + 3]};
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float* dst0 = ws + ((int64_t)w * EX_CHUNKS + c) * H * pstride + 8 + wv * JW;
    for (int idx = lane; idx < H * (JW / 4); idx += 64) {
        const int h = idx / (JW / 4), q = idx % (JW / 4);
        *(f32x4*)(dst0 + (int64_t)h * pstride + 4 * q) = *(const f32x4*)&Ol[h * OS + 4 * q];
    }
}

// (window, head): the EX_CHUNKS partials merged in chunk order and normalised:
// pen[w][h][j] = Σ_c e^(m_c - M) O_c[j] / Σ_c e^(m_c - M) l_c as an fp16 hi/lo pair
__global__ __launch_bounds__(256) void ex_merge_kernel(const float* __restrict__ ws, int pstride, int H, int D,
                                                       h16* __restrict__ pen, int64_t pen_lo,
                                                       const SelState* __restrict__ st) {
    const int w = blockIdx.x / H, h = blockIdx.x % H;
    if (st[w].done) return;
    const float cs2 = 1.4426950408889634f;
    const float* src = ws + ((int64_t)w * EX_CHUNKS * H + h) * pstride;
    float mc[EX_CHUNKS], e[EX_CHUNKS];
    float M = -INFINITY;
#pragma unroll
    for (int c = 0; c < EX_CHUNKS; ++c) {
        mc[c] = src[(int64_t)c * H * pstride];
        M = fmaxf(M, mc[c]);
    }
    float L = 0.f;
#pragma unroll
    for (int c = 0; c < EX_CHUNKS; ++c) {
        e[c] = __builtin_amdgcn_exp2f((mc[c] - M) * cs2);
        L = fmaf(src[(int64_t)c * H * pstride + 1], e[c], L);
    }
    const float inv = 1.0f / L;
    h16* out = pen + ((int64_t)w * H + h) * D;
    for (int j = threadIdx.x * 4; j < D; j += 256 * 4) {
        f32x4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < EX_CHUNKS; ++c) {
            const f32x4 v = *(const f32x4*)(src + (int64_t)c * H * pstride + 8 + j);
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = fmaf(v[i], e[c], a[i]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) split_h16(a[i] * inv, out, out + pen_lo, j + i);
    }
}

// kT[l][h][j][dd] = W[(2l)*D + h*64 + dd][j]: the K rows of each layer of dec.crosskv.w
__global__ __launch_bounds__(256) void ex_pack_kT_kernel(const h16* __restrict__ W, int L, int D,
                                                         h16* __restrict__ kT) {
    const int64_t n = (int64_t)L * D * D;
    const int H = D / 64;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const int dd = (int)(i % 64);
        const int64_t t = i / 64;
        const int j = (int)(t % D);
        const int64_t lh = t / D;
        const int h = (int)(lh % H), l = (int)(lh / H);
        kT[i] = W[((int64_t)(2 * l) * D + h * 64 + dd) * D + j];
    }
}
}  // namespace

bool exattn_supported(int D, int H) {
    if (H * 64 != D || H > 32) return false;
    return D == 1280 || D == 384 || D == 128 || D == 512 || D == 768 || D == 1024;
}

void launch_ex_pack_kT(const h16* W, int L, int D, h16* kT, hipStream_t s) {
    const int64_t n = (int64_t)L * D * D;
    ex_pack_kT_kernel<<<(unsigned)std::min<int64_t>((n + 255) / 256, 8192), 256, 0, s>>>(W, L, D, kT);
}

void launch_ex_qk(const float* part, int ks, const float* bias, int rows, int D, const h16* kT, h16* qp, int64_t qlo,
                  hipStream_t s) {
    const int H = D / 64;
    const int64_t slab = (int64_t)rows * D;
    ex_qk_kernel<<<dim3(H, D / 128), 256, 0, s>>>(part, ks, slab, bias, rows, D, kT, qp, qlo);
}

void launch_exattn(const h16* E, const h16* qp, int64_t qlo, int W, int T, int D, float* ws, int pstride,
                   h16* pen, int64_t pen_lo, const SelState* st, hipStream_t s) {
    const int H = D / 64;
    const unsigned grid = (unsigned)((W + 7) / 8 * 8 * EX_CHUNKS);
    switch (D) {
        case 1280: exattn_kernel<8, 160><<<grid, 512, 0, s>>>(E, qp, qlo, W, T, H, ws, pstride, st); break;
        case 1024: exattn_kernel<8, 128><<<grid, 512, 0, s>>>(E, qp, qlo, W, T, H, ws, pstride, st); break;
        case 768: exattn_kernel<8, 96><<<grid, 512, 0, s>>>(E, qp, qlo, W, T, H, ws, pstride, st); break;
        case 512: exattn_kernel<4, 128><<<grid, 256, 0, s>>>(E, qp, qlo, W, T, H, ws, pstride, st); break;
        case 384: exattn_kernel<4, 96><<<grid, 256, 0, s>>>(E, qp, qlo, W, T, H, ws, pstride, st); break;
        default: exattn_kernel<4, 32><<<grid, 256, 0, s>>>(E, qp, qlo, W, T, H, ws, pstride, st); break;
    }
    ex_merge_kernel<<<(unsigned)(W * H), 256, 0, s>>>(ws, pstride, H, D, pen, pen_lo, st);
}

}  // namespace osw
