// Decoder-step kernels (one token per window per step): self-attention over the
// KV cache, cross-attention over the 1500 precomputed encoder K/V, and the greedy
// token selection with Whisper's logits rules.
//
// Cross-attention is the bandwidth hot spot of decoding: each step reads the whole
// K and V of every (window, head): 2 x 1500 x 64 fp16 = 384 KB per (b, h).  One
// workgroup per (b, h); K rows are read 128 B per lane (8 x 16 B), V in 1 KiB
// contiguous wave-instructions (8 rows x 128 B), scores stay in LDS.
#include "decode.h"
#include "resln.h"

#include <climits>
#include <cstdio>
#include <cstdlib>

namespace osw {

namespace {
constexpr int HD = 64;
#include "selfattn.h"

// Sum the split-K partial slabs of a decoder projection for one (row, 64-column
// head slice) and round to fp16 (the GEMM output precision the oracle emulates).
// 256 threads: wave w sums slabs s = w, w+4, ... (independent loads in flight), then
// lane d adds the 4 wave sums in fixed order (deterministic).
__device__ __forceinline__ void reduce_head(const float* __restrict__ part, int ks, int64_t slab, int64_t off,
                                            const float* __restrict__ bias, int col, h16* dst, float* red4) {
    const int d = threadIdx.x & 63, w = threadIdx.x >> 6;
    float v = 0.f;
    int s = w;
    for (; s + 4 < ks; s += 8) v += part[s * slab + off + d] + part[(s + 4) * slab + off + d];
    if (s < ks) v += part[s * slab + off + d];
    red4[w * 64 + d] = v;
    __syncthreads();
    if (w == 0) {
        float r = bias ? bias[col + d] : 0.f;
        r += red4[d] + red4[64 + d] + red4[128 + d] + red4[192 + d];
        dst[d] = (h16)r;
    }
    __syncthreads();
}

// grid (H, B): q,k,v = Σ split-K partials of the fused qkv projection + bias; k,v
// appended to the cache at the device-side position; attend over 0..pos.  (Issuing the
// first K/V batch before the slab reduction left the batch-1 p50 unchanged, measured.)
// GATHER (beam rows): the row's ancestry is loaded before the slab reduction and staged in
// LDS behind its barrier, so it lands with the slabs (one round trip) instead of after.
template <bool GATHER, bool VPRE, bool KALL = false>
__global__ __launch_bounds__(256) void dec_self_attn_kernel(const float* __restrict__ part, int ks,
                                                            const float* __restrict__ bias, h16* __restrict__ kcache,
                                                            h16* __restrict__ vcache, const int* __restrict__ pos_ptr,
                                                            int H, int B, int ctx, h16* __restrict__ out,
                                                            int64_t lo_off, const int* __restrict__ anc, int group,
                                                            const SelState* __restrict__ st, int pos_row) {
    __shared__ h16 q16[HD];
    int h, b;
    if constexpr (GATHER) {
        // beam rows: the `group` hypotheses of one (window, head) run adjacently on one
        // XCD, so the cache rows they share through the ancestry table hit that L2
        const int nwg = gridDim.x, bid = blockIdx.x;
        const int qq = nwg / 8, rr = nwg % 8, xcd = bid % 8;
        const int lin = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + bid / 8;
        const int k = lin % group, w = lin / (group * H);
        h = (lin / group) % H;
        b = w * group + k;
    } else {
        h = blockIdx.x % H;
        b = blockIdx.x / H;
        // (selfattn.h: the batch-1 qkv GEMM's TAIL_ATTN runs the same function)
        self_attn_one<VPRE, false, KALL>(part, ks, bias, kcache, vcache, pos_ptr, H, B, ctx, out, lo_off, st, pos_row,
                                         b, h);
        return;
    }
    // every load of the prologue in one round trip: the row's state and position, its
    // ancestry (GATHER), the q/k/v slabs and bias
    const int done = st[b].done;
    const int D = H * HD;
    // graph replays may run past max_length on finished windows; pos_row: per-row counters (row refill)
    const int pos = min(pos_ptr[pos_row ? b : 0], ctx - 1);
    __shared__ int soff[GATHER ? 512 : 1];
    int an2[2];  // ancestry of keys tid and tid + 256 (ctx <= 448 < 512)
    if constexpr (GATHER) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int key = threadIdx.x + 256 * i;
            an2[i] = anc[(int64_t)b * ctx + min(key, ctx - 1)];
        }
    }
    const int64_t slab = (int64_t)B * 3 * D, row = (int64_t)b * 3 * D;
    QkvLoad L;
    qkv_load(part, ks, slab, row, D, h, bias, L);
    // a finished row (its <|endoftext|> is chosen; graph replays keep stepping it until
    // the whole batch is done) writes nothing and reads nothing more: its outputs are never used
    if (done) return;
    h16* kc = kcache + ((int64_t)b * H + h) * ctx * HD;
    h16* vc = vcache + ((int64_t)b * H + h) * ctx * HD;
    qkv_finish(part, ks, slab, row, D, h, L, q16, kc + (int64_t)pos * HD, vc + (int64_t)pos * HD);
    if constexpr (GATHER) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int key = threadIdx.x + 256 * i;
            soff[key] = key < pos ? an2[i] - b : 0;  // the newest key (pos) is this row's own
        }
    }
    __threadfence_block();
    __syncthreads();
    if constexpr (GATHER)
        attend_one<448, true, false, VPRE>(q16, kc, vc, pos + 1, out + (int64_t)b * D + h * HD, lo_off, soff,
                                           (int64_t)H * ctx * HD);
    else
        attend_one<448, false, true, VPRE>(q16, kc, vc, pos + 1, out + (int64_t)b * D + h * HD, lo_off);
}

// grid H*B (flattened): q = Σ split-K partials of the cross-attention q projection
// + bias; row b attends window b / beam: K at ((w*H + h)*T*64) of xk, V likewise.
// Workgroups are remapped XCD-contiguously with the beam rows of one (window, head)
// adjacent, so those rows' reads of the same 384 KB K/V share one L2.
__global__ __launch_bounds__(256) void dec_cross_attn_kernel(const float* __restrict__ part, int ks,
                                                             const float* __restrict__ bias,
                                                             const h16* __restrict__ xk, const h16* __restrict__ xv,
                                                             int H, int B, int T, int beam, h16* __restrict__ out,
                                                             int64_t lo_off) {
    __shared__ h16 q16[HD];
    __shared__ float red4[256];
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int qq = nwg / 8, rr = nwg % 8, xcd = bid % 8;
    const int lin = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + bid / 8;
    const int k = lin % beam, h = (lin / beam) % H, w = lin / (beam * H);
    const int b = w * beam + k;
    const int D = H * HD;
    reduce_head(part, ks, (int64_t)B * D, (int64_t)b * D + h * HD, bias, h * HD, q16, red4);
    const int64_t hoff = ((int64_t)w * H + h) * T * HD;
    attend_one<1536>(q16, xk + hoff, xv + hoff, T, out + (int64_t)b * D + h * HD, lo_off);
}

// ---------------------------------------------------------------------------
// Cross-attention split over fixed key chunks (flash-decoding).  The T = 1500 keys
// of a (window, head) are cut into XCH = 8 fixed chunks of <= 192 keys; one
// workgroup per (window, head, chunk) serves all `beam` decoder rows of the window.
// Every lane first issues its 6 K and 6 V row pieces (12 x 16 B; 48 KB per
// workgroup, the whole chunk in one HBM round trip), then reduces the rows' q from
// the q projection's split-K slabs while the loads land.  Per row it writes the
// chunk max m, l = Σ exp(s - m) and the unnormalised Σ exp(s - m)·v to a workspace
// with device-scope stores (they write through the XCD's L2; a release fence would
// write back the whole L2 instead, measured 7x slower at 64 windows) and takes an
// arrival ticket; the last of the 8 chunk workgroups of a (window, head) merges them
// in fixed chunk order, so the output does not depend on the batch size, dispatch
// order or XCD placement, and no separate merge launch is needed.  Small
// batches get 8x the workgroups of one-per-(row, head) (B = 1: 160 instead of 20),
// and beam rows read each K/V chunk once instead of once per row.
// Lane map: kg = tid >> 3 (32 key groups), c = tid & 7 (dims 8c..8c+7); the lane
// holds keys u*32 + kg (u = 0..5) of the chunk for both scores and P·V.  K/V loads are
// nontemporal (1.97 GB per step at 64 windows cannot stay in the 256 MB MALL): 90 -> 84 us.
constexpr int XCH = XCHUNKS, XKEYS = 192, XU = XKEYS / 32;
static_assert(XCH == 8, "the (window, head) -> XCD map assumes 8 chunks");

// merge of a (window, head)'s chunk partials in fixed chunk order: out = Σ e^(m_s - M) acc_s /
// Σ e^(m_s - M) l_s (device-scope loads: the other chunks' partials may come from another
// XCD's writes); beam rows are spread over the 4 waves so their load round trips overlap
__device__ __forceinline__ void xattn_merge(const float* __restrict__ ws, int r0, int beam, int H, int h,
                                            h16* __restrict__ out, int64_t lo_off) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, D = H * HD;
    for (int k = wv; k < beam; k += 4) {
        const float* src = ws + ((int64_t)(r0 + k) * H + h) * XCH * XPART;
        float mm[XCH];
        float M = -INFINITY;
#pragma unroll
        for (int q = 0; q < XCH; ++q) {
            mm[q] = __hip_atomic_load(src + q * XPART, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            M = fmaxf(M, mm[q]);
        }
        float L = 0.f, O = 0.f;
#pragma unroll
        for (int q = 0; q < XCH; ++q) {
            const float e = __expf(mm[q] - M);
            L = fmaf(__hip_atomic_load(src + q * XPART + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), e, L);
            O = fmaf(__hip_atomic_load(src + q * XPART + 4 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), e, O);
        }
        split_h16(O / L, out, out + lo_off, (int64_t)(r0 + k) * D + h * HD + lane);
    }
}

// LDS writes of every wave visible, without draining the wave's outstanding global loads
// (__syncthreads waits for vmcnt(0) too)
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

typedef __fp16 fp16x4_t __attribute__((__vector_size__(4 * sizeof(__fp16))));
__device__ __forceinline__ h16x4 ds_read_tr(const h16* p) {  // ds_read_b64_tr_b16 (as attn.hip)
    fp16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4f16((OSW_LDS fp16x4_t*)p);
    return __builtin_bit_cast(h16x4, v);
}

template <int NB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NB > 5 ? 4 : NB > 1 ? 5 : 1))) void dec_xattn_chunk_kernel(const float* __restrict__ part, int ks,
                                                              const float* __restrict__ bias,
                                                              const h16* __restrict__ xk, const h16* __restrict__ xv,
                                                              int H, int W, int T, int beam, float* __restrict__ ws,
                                                              int* __restrict__ ticket, h16* __restrict__ out,
                                                              int64_t lo_off, const SelState* __restrict__ st) {
    __shared__ float red[4][NB][HD];
    __shared__ __attribute__((aligned(16))) float pvs[NB > 1 ? 4 : 1][8][HD];  // beam rows' P·V reduction image
    __shared__ float rm[4][NB], rl[4][NB];
    __shared__ float qsh[NB][HD];
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, kg = tid >> 3, c = tid & 7;
    const int bid = blockIdx.x;
    const int chunk = (bid >> 3) & 7;
    const int p = (bid & 7) + 8 * (bid >> 6);  // (window, head) pair; its 8 chunks share one XCD (bid % 8)
    if (p >= W * H) return;
    const int h = p % H, w = p / H;
    // a window whose rows are all finished skips its 384 KB of K/V per head (the 8 chunk
    // workgroups of a (window, head) read the same flags, so none of them takes a ticket)
    {
        int done = 1;  // every flag loaded at once (no short-circuit chain of dependent loads)
#pragma unroll
        for (int k = 0; k < NB; ++k)
            if (k < beam) done &= st[w * beam + k].done;
        if (done) return;
    }
    const int D = H * HD;
    const int per = (T + XCH - 1) / XCH;
    const int k0 = chunk * per, nk = min(T, k0 + per) - k0;
    const int64_t hoff = ((int64_t)w * H + h) * T * HD;
    // q of row r0 + k: fp16(bias + Σ split-K partials) / sqrt(64), the order of reduce_head
    // (wave wv: slabs wv, wv+4 pairwise by 8).  With ks <= 8 the wave's two slabs and the
    // bias are issued before the K/V stream, so the q reduction waits for them alone.
    const int r0 = w * beam;
    const int64_t slab = (int64_t)W * beam * D;
    const float bq = bias[h * HD + lane];
    float qa[NB], qb[NB];
    if (ks <= 8) {
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            const int64_t off = (int64_t)(r0 + min(k, beam - 1)) * D + h * HD + lane;
            qa[k] = part[min(wv, ks - 1) * slab + off];
            qb[k] = part[min(wv + 4, ks - 1) * slab + off];
        }
    }
    h16x8 kf[XU], vf[XU];
#pragma unroll
    for (int u = 0; u < XU; ++u) {
        const int key = k0 + min(u * 32 + kg, nk - 1);
        kf[u] = __builtin_nontemporal_load((const h16x8*)(xk + hoff + (int64_t)key * HD + 8 * c));
        vf[u] = __builtin_nontemporal_load((const h16x8*)(xv + hoff + (int64_t)key * HD + 8 * c));
    }
#pragma unroll
    for (int k = 0; k < NB; ++k) {
        if (k >= beam) break;
        float v = 0.f;
        if (ks <= 8) {
            if (wv + 4 < ks) v += qa[k] + qb[k];
            else if (wv < ks) v += qa[k];
        } else {
            const int64_t off = (int64_t)(r0 + k) * D + h * HD + lane;
            int s = wv;
            for (; s + 4 < ks; s += 8) v += part[s * slab + off] + part[(s + 4) * slab + off];
            if (s < ks) v += part[s * slab + off];
        }
        red[wv][k][lane] = v;
    }
    __syncthreads();
    if (wv == 0) {
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            if (k >= beam) break;
            float r = bq;
            r += red[0][k][lane] + red[1][k][lane] + red[2][k][lane] + red[3][k][lane];
            qsh[k][lane] = (float)(h16)r * 0.125f;
        }
    }
    __syncthreads();
    // scores (8 lanes per key, combined by 3 xor-shuffles) and the chunk max per row
    float sc[NB][XU], mx[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
        mx[k] = -INFINITY;
        if (k >= beam) continue;
        // beam rows (VALU-bound, §5.5): q/8 in fp16 and 4 v_dot2_f32_f16 per score instead
        // of 8 conversions + 8 FMAs.  fp16(q)/8 is exact while |q| >= 2^-11 (q/8 stays a
        // normal fp16); smaller elements lose low mantissa bits, an error below 2^-25
        // absolute per product, far inside the fp32 sums' own rounding.  (Scaling the
        // fp32 dot instead costs one more VALU op per score in this VALU-bound kernel:
        // 122 -> 130 us per launch, measured.)
        float q[8];
        h16x2 q2[4];
#pragma unroll
        for (int i = 0; i < 8; ++i) q[i] = qsh[k][8 * c + i];
#pragma unroll
        for (int i = 0; i < 4; ++i) q2[i] = h16x2{(h16)q[2 * i], (h16)q[2 * i + 1]};
#pragma unroll
        for (int u = 0; u < XU; ++u) {
            float d = 0.f;
            if constexpr (NB > 1) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    d = __builtin_amdgcn_fdot2(h16x2{kf[u][2 * i], kf[u][2 * i + 1]}, q2[i], d, false);
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) d = fmaf((float)kf[u][i], q[i], d);
            }
            d += xor_lane<1>(d);
            d += xor_lane<2>(d);
            d += xor_lane<4>(d);
            sc[k][u] = d;
            if (u * 32 + kg < nk) mx[k] = fmaxf(mx[k], d);
        }
        mx[k] = wave_max(mx[k]);
        if (lane == 0) rm[wv][k] = mx[k];
    }
    __syncthreads();
    // p = exp(s - m) (0 past the chunk end); l = Σ p (one lane per key); P·V per lane
    float acc[NB][8], ls[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
        ls[k] = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[k][e] = 0.f;
        if (k >= beam) continue;
        const float m = fmaxf(fmaxf(rm[0][k], rm[1][k]), fmaxf(rm[2][k], rm[3][k]));
        mx[k] = m;
#pragma unroll
        for (int u = 0; u < XU; ++u) {
            const float pu = u * 32 + kg < nk ? __expf(sc[k][u] - m) : 0.f;
            ls[k] += pu;
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[k][e] = fmaf(pu, (float)vf[u][e], acc[k][e]);
        }
        // the 8 key groups of this wave: lanes c + 8 kr, kr = 0..7, summed in the order
        // ((0+1)+(2+3))+((4+5)+(6+7)).  Beam rows (VALU-bound) go through a per-wave LDS
        // image (2 stores + 8 loads per lane) instead of 24 shuffle-adds per row.
        if constexpr (NB > 1) {
            float* t = &pvs[wv][lane >> 3][8 * c];
            *(f32x4*)t = f32x4{acc[k][0], acc[k][1], acc[k][2], acc[k][3]};
            *(f32x4*)(t + 4) = f32x4{acc[k][4], acc[k][5], acc[k][6], acc[k][7]};
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            float tv[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) tv[r] = pvs[wv][r][lane];
            red[wv][k][lane] = ((tv[0] + tv[1]) + (tv[2] + tv[3])) + ((tv[4] + tv[5]) + (tv[6] + tv[7]));
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                float a = acc[k][e];
                a += xor_lane<8>(a);
                a += xor_lane<16>(a);
                a += xor_lane<32>(a);
                acc[k][e] = a;
            }
            if (lane < 8) {
#pragma unroll
                for (int e = 0; e < 8; ++e) red[wv][k][8 * c + e] = acc[k][e];
            }
        }
        float l = c == 0 ? ls[k] : 0.f;
        l = wave_sum(l);
        if (lane == 0) rl[wv][k] = l;
    }
    __syncthreads();
    __shared__ int last;
    if (wv == 0) {
        // publish this chunk's partials with device-scope (write-through) stores, wait for
        // them, then take the (window, head) arrival ticket: the 8th arriver merges
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            if (k >= beam) break;
            float* dst = ws + (((int64_t)(r0 + k) * H + h) * XCH + chunk) * XPART;
            const float a = (red[0][k][lane] + red[1][k][lane]) + (red[2][k][lane] + red[3][k][lane]);
            const float l = (rl[0][k] + rl[1][k]) + (rl[2][k] + rl[3][k]);
            __hip_atomic_store(dst + 4 + lane, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (lane == 0) {
                __hip_atomic_store(dst, mx[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(dst + 1, l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __builtin_amdgcn_s_waitcnt(0);  // the stores above are complete at device scope
        int old = 0;
        if (lane == 0) old = __hip_atomic_fetch_add(ticket + p, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        old = __builtin_amdgcn_readfirstlane(old);
        if (lane == 0) {
            last = old == XCH - 1;
            if (old == XCH - 1) __hip_atomic_store(ticket + p, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (NB == 1 && wv != 0) return;  // one row: wave 0 merges alone
    __syncthreads();
    if (!last) return;
    xattn_merge(ws, r0, beam, H, h, out, lo_off);
}

// Beam rows (2..8 per window): dec_xattn_chunk_kernel's (window, head, key chunk)
// decomposition, partials and last-arriver merge, with the scores and P·V on MFMA (the
// VALU form ran VALU-bound: 120 us per launch at 64 windows x 5 beams against 84 us for
// the greedy rows' identical K/V bytes).  The window's rows are the 16 MFMA columns
// (rows >= beam: q = 0, results unused).
//   Sᵀ = K·Qᵀ   v_mfma_f32_16x16x32_f16; A = K rows straight from HBM (lane: key 16t + li,
//               dims 32s + 8g .. +8, one 16-B piece), B = fp16(q) (the q the VALU forms
//               use, unscaled; the exact 1/8 is applied to the fp32 scores)
//   Oᵀ = Vᵀ·Pᵀ  v_mfma_f32_16x16x16_f16; A = V staged in LDS (swizzled rows), read with
//               ds_read_b64_tr_b16 (the encoder attention's transposed read); B = P in the
//               score registers as an fp16 hi/lo pair, two MFMAs, so P keeps ~22 bits as in
//               the fp32 VALU form
// Wave w: keys 48w .. 48w+47 (3 tiles of 16) for the scores and for P·V over all 64 dims
// (one max for the workgroup, exchanged before the exponentials); the 4 waves' P·V sums
// meet in LDS in fixed order.
// KLDS: K arrives like V, 8 rows x 128 B per wave-instruction (whole cache lines), and is
// staged through the V image into the MFMA A layout; otherwise each lane loads its A
// fragment straight from HBM (16 keys x 64 B per wave-instruction: every line is touched
// by two instructions, the pattern that streamed the logits matrix at 3.95 instead of
// 5.4 TB/s, tools/gemv_probe.hip).  Same K elements in the same fragments: same results.
template <int NB, bool KLDS = true>
__global__ __launch_bounds__(256) void dec_xattn_mfma_kernel(const float* __restrict__ part, int ks,
                                                             const float* __restrict__ bias,
                                                             const h16* __restrict__ xk, const h16* __restrict__ xv,
                                                             int H, int W, int T, int beam, float* __restrict__ ws,
                                                             int* __restrict__ ticket, h16* __restrict__ out,
                                                             int64_t lo_off, const SelState* __restrict__ st) {
    static_assert(NB <= 16 && XKEYS == 192, "16 MFMA columns; 4 waves x 3 key tiles");
    __shared__ __attribute__((aligned(16))) h16 Vl[XKEYS * HD];
    __shared__ __attribute__((aligned(16))) h16 qsh[16][HD];
    __shared__ float red[4][NB][HD];
    __shared__ float rm[4][16], rl[4][16], bsh[4][HD];
    __shared__ int last;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, g = lane >> 4, li = lane & 15;
    const int bid = blockIdx.x;
    const int chunk = (bid >> 3) & 7;
    const int p = (bid & 7) + 8 * (bid >> 6);  // (window, head); its 8 chunks share one XCD
    if (p >= W * H) return;
    const int h = p % H, w = p / H;
    {
        int done = 1;
#pragma unroll
        for (int k = 0; k < NB; ++k)
            if (k < beam) done &= st[w * beam + k].done;
        if (done) return;
    }
    const int D = H * HD;
    const int per = (T + XCH - 1) / XCH;
    const int k0 = chunk * per, nk = min(T, k0 + per) - k0;
    const int64_t hoff = ((int64_t)w * H + h) * T * HD;
    // q of row r0 + k: fp16(bias + Σ split-K partials), the VALU kernel's order (ks <= 8:
    // wave wv holds slabs wv and wv + 4).  The slab loads go out first and all at once;
    // the K/V loads follow, and the barriers before the scores are raw s_barriers: vmcnt
    // retires loads in issue order, so the q reduction waits for its own loads only,
    // never for the 48 KB of K/V behind them (a __syncthreads would drain them all).
    const int r0 = w * beam;
    const int64_t slab = (int64_t)W * beam * D;
    float qa[NB], qb[NB];
    const float bq = bias[h * HD + lane];
#pragma unroll
    for (int k = 0; k < NB; ++k) {
        const int64_t off = (int64_t)(r0 + min(k, beam - 1)) * D + h * HD + lane;
        qa[k] = part[min(wv, ks - 1) * slab + off];
        qb[k] = part[min(wv + 4, ks - 1) * slab + off];
    }
    // K fragments of this wave's 3 key tiles (A operand), nontemporal, clamped to the chunk
    h16x8 kf[3][2], kr[6];
    if constexpr (KLDS) {
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const int r = (i * 4 + wv) * 8 + (lane >> 3);
            kr[i] = __builtin_nontemporal_load((const h16x8*)(xk + hoff + (int64_t)(k0 + min(r, nk - 1)) * HD + 8 * (lane & 7)));
        }
    } else {
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const int key = k0 + min(16 * (3 * wv + t) + li, nk - 1);
#pragma unroll
            for (int s = 0; s < 2; ++s)
                kf[t][s] = __builtin_nontemporal_load((const h16x8*)(xk + hoff + (int64_t)key * HD + 32 * s + 8 * g));
        }
    }
    // V chunk: 24 pieces of 8 rows x 128 B, 6 per wave, into registers now and into LDS
    // (16-B chunk XOR-swizzled by row) once they land.  Plain loads, not global_load_lds:
    // with LDS-DMA in flight hipcc drains vmcnt(0) before any use of an earlier load.
    h16x8 vr[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const int r = (i * 4 + wv) * 8 + (lane >> 3);
        vr[i] = __builtin_nontemporal_load((const h16x8*)(xv + hoff + (int64_t)(k0 + min(r, nk - 1)) * HD + 8 * (lane & 7)));
    }
    const bool has_a = wv < ks, has_b = wv + 4 < ks;
#pragma unroll
    for (int k = 0; k < NB; ++k) red[wv][k][lane] = (has_a ? qa[k] : 0.f) + (has_b ? qb[k] : 0.f);
    bsh[wv][lane] = bq;  // every wave, through LDS: hipcc cannot sink the load past the K/V loads
    if constexpr (KLDS) {
        // the K chunk into the V image (V goes there after the scores: the max exchange's
        // barrier below orders every wave's fragment reads before the V stores)
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const int r = (i * 4 + wv) * 8 + (lane >> 3);
            *(h16x8*)&Vl[r * HD + (((lane & 7) ^ ((r >> 1) & 7)) * 8)] = kr[i];
        }
    }
    lds_barrier();
    if (wv == 0) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            h16 q = (h16)0.f;
            if (k < beam && k < NB) {
                float r = bsh[0][lane];
                r += red[0][k][lane] + red[1][k][lane] + red[2][k][lane] + red[3][k][lane];
                q = (h16)r;
            }
            qsh[k][lane] = q;
        }
    }
    lds_barrier();
    const h16x8 qf0 = *(const h16x8*)&qsh[li][8 * g], qf1 = *(const h16x8*)&qsh[li][32 + 8 * g];
    if constexpr (KLDS) {
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const int r = 16 * (3 * wv + t) + li;
#pragma unroll
            for (int s = 0; s < 2; ++s) kf[t][s] = *(const h16x8*)&Vl[r * HD + (((4 * s + g) ^ ((r >> 1) & 7)) * 8)];
        }
    }
    // scores: lane holds key 16(3wv + t) + 4g + i of row li
    f32x4 sc[3];
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 3; ++t) {
        f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
        a = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[t][0], qf0, a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[t][1], qf1, a, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int key = 16 * (3 * wv + t) + 4 * g + i;
            a[i] = key < nk ? a[i] * 0.125f : -INFINITY;
            mx = fmaxf(mx, a[i]);
        }
        sc[t] = a;
    }
    mx = fmaxf(mx, xor_lane<16>(mx));
    mx = fmaxf(mx, xor_lane<32>(mx));
    if (g == 0) rm[wv][li] = mx;
    lds_barrier();
    const float m = fmaxf(fmaxf(rm[0][li], rm[1][li]), fmaxf(rm[2][li], rm[3][li]));
    // p = exp(s - m) as an fp16 hi/lo pair in the score registers, which are already the
    // B operand of v_mfma_f32_16x16x16_f16 (lane: keys 4g .. 4g+3 of a tile, row li)
    float ls = 0.f;
    h16x4 ph[3], pl[3];
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float pv = __expf(sc[t][i] - m);
            ls += pv;
            ph[t][i] = (h16)pv;
            pl[t][i] = (h16)(pv - (float)ph[t][i]);
        }
    ls += xor_lane<16>(ls);
    ls += xor_lane<32>(ls);
    if (g == 0) rl[wv][li] = ls;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const int r = (i * 4 + wv) * 8 + (lane >> 3);
        *(h16x8*)&Vl[r * HD + (((lane & 7) ^ ((r >> 1) & 7)) * 8)] = vr[i];
    }
    __syncthreads();
    // P·V over this wave's 48 keys, all 64 dims: Oᵀ += Vᵀ·Pᵀ, A = V by ds_read_b64_tr_b16
    // (lane: dim 16dt + li, keys 4g .. 4g+3 of the tile); lane ends with O[li][16dt + 4g + i]
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    {
        const int q4 = li >> 2, p4 = li & 3;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const int ra = 48 * wv + 16 * t + 4 * g + q4;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                const int col = 16 * dt + 4 * p4;
                const h16x4 va = ds_read_tr(&Vl[ra * HD + (((col >> 3) ^ ((ra >> 1) & 7)) * 8) + (col & 7)]);
                o[dt] = __builtin_amdgcn_mfma_f32_16x16x16f16(va, ph[t], o[dt], 0, 0, 0);
                o[dt] = __builtin_amdgcn_mfma_f32_16x16x16f16(va, pl[t], o[dt], 0, 0, 0);
            }
        }
    }
    // the 4 waves' key ranges summed in fixed order through LDS (red is free again)
    if (li < beam && li < NB) {
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) *(f32x4*)&red[wv][li][16 * dt + 4 * g] = o[dt];
    }
    __syncthreads();
    if (wv == 0) {
        // publish (m, l, Σp·v) with device-scope (write-through) stores, wait for them, then
        // the (window, head) arrival ticket: the 8th arriver merges
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            if (k >= beam) break;
            float* dst = ws + (((int64_t)(r0 + k) * H + h) * XCH + chunk) * XPART;
            const float a = (red[0][k][lane] + red[1][k][lane]) + (red[2][k][lane] + red[3][k][lane]);
            __hip_atomic_store(dst + 4 + lane, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (lane == 0) {
                const float mk = fmaxf(fmaxf(rm[0][k], rm[1][k]), fmaxf(rm[2][k], rm[3][k]));
                __hip_atomic_store(dst, mk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(dst + 1, (rl[0][k] + rl[1][k]) + (rl[2][k] + rl[3][k]), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __builtin_amdgcn_s_waitcnt(0);
        int old = 0;
        if (lane == 0) old = __hip_atomic_fetch_add(ticket + p, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        old = __builtin_amdgcn_readfirstlane(old);
        if (lane == 0) {
            last = old == XCH - 1;
            if (old == XCH - 1) __hip_atomic_store(ticket + p, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    if (!last) return;
    xattn_merge(ws, r0, beam, H, h, out, lo_off);
}

// grid B, 256 threads: x[b] += bias + Σ split-K partials (residual stream, fp32), then
// LayerNorm(x[b]) -> y[b] as an fp16 pair (the next projection's operand); with
// part == nullptr the embedding entry x[b] = tok_emb[tok[b]] + pos_emb[pos].  The
// arithmetic is resln_rows (resln.h), shared with the fused GEMM prologue.
__global__ __launch_bounds__(256) void dec_resid_ln_kernel(ResLnArgs A, h16* __restrict__ y, int64_t lo_off) {
    __shared__ __attribute__((aligned(16))) float red[resln_scratch(1, 1280)];
    const int b = blockIdx.x;
    resln_rows<1, 8, true>(A, b, 1, true, red,
                  [&](int, int c, float v) { split_h16(v, y, y + lo_off, (int64_t)b * A.D + c); });
}

// fc1: h[b][n] = fp16 pair of gelu(bias + Σ partials) (gelu_reduce_one, shared with the
// fused fc2 prologue)
__global__ __launch_bounds__(256) void dec_reduce_gelu_kernel(const float* __restrict__ part, int ks, int64_t total,
                                                              int N, const float* __restrict__ bias,
                                                              h16* __restrict__ y, int64_t lo_off) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
        split_h16(gelu_reduce_one(part, ks, total, bias, i, (int)(i % N)), y, y + lo_off, i);
}

#include "select.h"

// ---------------------------------------------------------------------------
// Beam search candidates (restated CTranslate2 BeamSearch, see oracle/decode.py).
struct BeamCand {
    float s;
    int i;  // beam_slice_body: (raw logit, token id); beam_update: (score, beam slot * V + token)
};
constexpr int BEAM_SLICES = SEL_SPLIT;  // vocabulary slices per row (one pass: the select slices)
constexpr int TOPK_VPT = 16;            // logits one thread holds
constexpr int MAXK2 = 2 * MAX_BEAM;
static_assert(BEAM_SLICES * 256 * TOPK_VPT >= SEL_SPLIT * 4096, "osw.hip admits V <= SEL_SPLIT * 4096: one batch per slice");

// Ordered keys for the candidate ranking.  score_key: a float as an int with the same
// order (-0 as +0, NaN excluded by the callers); an involution, so score_of reads the float
// back.  rank_key: (score desc, id asc) as one unsigned 64-bit key (0: none).
// wave_max_key: the wave's largest int in every lane -- row shifts 1, 2, 4, 8 (lane 15 of
// each row holds the row's maximum), row broadcasts 15 and 31, lane 63 read back.
__device__ __forceinline__ int score_key(float v) {
    const int u = __float_as_int(v == 0.f ? 0.f : v);
    return u ^ ((u >> 31) & 0x7fffffff);
}
__device__ __forceinline__ float score_of(int k) { return __int_as_float(k ^ ((k >> 31) & 0x7fffffff)); }
__device__ __forceinline__ unsigned long long rank_key(float v, int id) {
    return ((unsigned long long)((unsigned)score_key(v) ^ 0x80000000u) << 32) | (unsigned)~id;
}
__device__ __forceinline__ int wave_max_key(int t) {
    t = max(t, __builtin_amdgcn_update_dpp(INT_MIN, t, 0x111, 0xf, 0xf, false));  // row_shr:1
    t = max(t, __builtin_amdgcn_update_dpp(INT_MIN, t, 0x112, 0xf, 0xf, false));  // row_shr:2
    t = max(t, __builtin_amdgcn_update_dpp(INT_MIN, t, 0x114, 0xf, 0xf, false));  // row_shr:4
    t = max(t, __builtin_amdgcn_update_dpp(INT_MIN, t, 0x118, 0xf, 0xf, false));  // row_shr:8
    t = max(t, __builtin_amdgcn_update_dpp(INT_MIN, t, 0x142, 0xa, 0xf, false));  // row_bcast:15
    t = max(t, __builtin_amdgcn_update_dpp(INT_MIN, t, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return __builtin_amdgcn_readlane(t, 63);
}
// rank of this lane's key among lanes [0, n) of the wave (n <= 64, wave-uniform; lanes
// [n, 64) hold key 0, so the walk runs in groups of 4 lanes)
__device__ __forceinline__ int wave_rank(unsigned long long key, int n) {
    const unsigned klo = (unsigned)key, khi = (unsigned)(key >> 32);
    int rank = 0;
    for (int j = 0; j < n; j += 4) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const unsigned long long f = ((unsigned long long)__builtin_amdgcn_readlane(khi, j + q) << 32) |
                                         (unsigned)__builtin_amdgcn_readlane(klo, j + q);
            rank += f > key ? 1 : 0;
        }
    }
    return rank;
}

// A beam row's sampling step, one vocabulary slice, ONE pass over its logits: the slice
// statistics of select_partial_body (same entries in the same order, so the same
// SelPart) and two candidate lists for beam_update: the slice's top 2*beam tokens by raw
// logit among the rule-allowed tokens (list A, used when text is allowed) and among the
// allowed timestamps (list B, used when the timestamp-mass rule suppresses text), each
// followed by -inf fillers in token order.  Within a row every candidate's score is
// sum_lp + (x - lse) with one lse per list, monotonic in x, so beam_update ranks these
// exactly as the former separate top-k pass ranked the scores (score desc, flat index
// asc).  Two known divergences from ranking the rounded scores: a row whose sum_lp is
// already -inf (all scores tie at -inf), and two different logits whose scores round to
// the same float at the top-2K cutoff (here the larger logit wins, there the lower flat
// index); CTranslate2's tie order on such inputs is unpinned (no fixture covers it).
//
// FAST (default): the K2 pops (a block barrier each) run only where a cheaper exact form
// cannot: each wave finds the K2-th largest of its 64 lane maxima (wave-only pops, no
// barrier), T = the largest of the 4.  At least K2 allowed entries are >= T (the popped
// lanes' maxima), so the slice's top K2 lie in S = {allowed live entries >= T}; S is
// gathered in LDS and each member's rank under (key desc, token asc) -- the pops' order --
// is counted directly.  Falls back to the pops when T = -inf (fewer than K2 finite
// allowed entries in every wave) or |S| > 256.
template <bool FAST>
__device__ __forceinline__ void beam_slice_body(const float* __restrict__ logits, const SelParams& P, int step,
                                                const unsigned* __restrict__ supmask, const SelState& s,
                                                SelPart* __restrict__ parts, BeamCand* __restrict__ cand) {
    __shared__ ArgMax red[2][4];
    __shared__ SelPart wp[4];
    const int b = blockIdx.x, sl = blockIdx.y, tid = threadIdx.x;
    const int K2 = 2 * P.beam;
    BeamCand* outA = cand + ((int64_t)b * BEAM_SLICES + sl) * 2 * MAXK2;
    BeamCand* outB = outA + MAXK2;
    const int per = (P.V + SEL_SPLIT - 1) / SEL_SPLIT;
    const int lo = sl * per, hi = min(P.V, lo + per);
    const float* x = logits + (int64_t)b * P.V;
    float xv[TOPK_VPT];
    unsigned mw[TOPK_VPT];
#pragma unroll
    for (int u = 0; u < TOPK_VPT; ++u) {
        const int v = min(lo + u * 256 + tid, hi - 1);
        xv[u] = x[v];
        mw[u] = supmask[v >> 5];
    }
    const RowRules R = row_rules(P, s);
    float m_all = -INFINITY, s_all = 0.f, m_ts = -INFINITY, s_ts = 0.f;
    ArgMax a_all{-INFINITY, 0x7fffffff}, a_text{-INFINITY, 0x7fffffff}, a_ts{-INFINITY, 0x7fffffff};
    unsigned okA = 0, okB = 0, live = 0;  // allowed / allowed timestamp / in slice and not NaN
#pragma unroll
    for (int u = 0; u < TOPK_VPT; ++u) {
        const int v = lo + u * 256 + tid;
        if (v >= hi) continue;
        if (xv[u] == xv[u]) live |= 1u << u;
        if (tok_masked_w(P, R, mw[u], v)) continue;
        const float xu = xv[u];
        lse_add(m_all, s_all, xu);
        a_all = amax(a_all, ArgMax{xu, v});
        okA |= 1u << u;
        if (v >= P.tb) {
            lse_add(m_ts, s_ts, xu);
            a_ts = amax(a_ts, ArgMax{xu, v});
            okB |= 1u << u;
        } else {
            a_text = amax(a_text, ArgMax{xu, v});
        }
    }
    {  // the slice statistics, merged exactly as select_partial_body merges them
        auto merge = [&](auto o) {
            constexpr int O = decltype(o)::value;
            lse_merge(m_all, s_all, xor_lane<O>(m_all), xor_lane<O>(s_all));
            lse_merge(m_ts, s_ts, xor_lane<O>(m_ts), xor_lane<O>(s_ts));
            a_all = amax(a_all, ArgMax{xor_lane<O>(a_all.v), xor_lane<O>(a_all.i)});
            a_text = amax(a_text, ArgMax{xor_lane<O>(a_text.v), xor_lane<O>(a_text.i)});
            a_ts = amax(a_ts, ArgMax{xor_lane<O>(a_ts.v), xor_lane<O>(a_ts.i)});
        };
        merge(IC<32>{}), merge(IC<16>{}), merge(IC<8>{}), merge(IC<4>{}), merge(IC<2>{}), merge(IC<1>{});
        if ((tid & 63) == 0)
            wp[tid >> 6] = SelPart{m_all, s_all, m_ts, s_ts, a_all.v, a_text.v, a_ts.v, a_all.i, a_text.i, a_ts.i};
    }
    // top K2 of one list by (key desc, token asc); key = x if allowed, else -inf
    auto pops = [&](unsigned ok, BeamCand* out) {
        unsigned used = ~live;
        auto best = [&]() {
            int bu = -1;
            float bv = -INFINITY;
#pragma unroll
            for (int u = 0; u < TOPK_VPT; ++u) {
                const float k = ((ok >> u) & 1u) ? xv[u] : -INFINITY;
                if (!((used >> u) & 1u) && (bu < 0 || k > bv)) { bv = k; bu = u; }
            }
            return bu < 0 ? ArgMax{-INFINITY, INT_MAX} : ArgMax{bv, lo + bu * 256 + tid};
        };
        // pop the block-wide best K2 times (wave DPP argmax + one LDS exchange per pop; only
        // the owner of a popped entry rescans).  (Each wave popping its own top K2 and wave 0
        // merging the 4*K2 survivors, with no barrier per pop, measured 116 vs 101 us at 320 rows.)
        ArgMax mine = best();
        for (int r = 0; r < K2; ++r) {
            ArgMax a = mine;
            auto stp = [&](auto o) {
                constexpr int O = decltype(o)::value;
                a = amax(a, ArgMax{xor_lane<O>(a.v), xor_lane<O>(a.i)});
            };
            stp(IC<32>{}), stp(IC<16>{}), stp(IC<8>{}), stp(IC<4>{}), stp(IC<2>{}), stp(IC<1>{});
            if ((tid & 63) == 0) red[r & 1][tid >> 6] = a;
            __syncthreads();
            ArgMax g = red[r & 1][0];
#pragma unroll
            for (int w = 1; w < 4; ++w) g = amax(g, red[r & 1][w]);
            if (tid == 0) out[r] = BeamCand{g.v, g.i};
            if (g.i != INT_MAX && mine.i == g.i) {
                used |= 1u << ((g.i - lo - tid) >> 8);
                mine = best();
            }
        }
    };
    constexpr int SCAP = 256;
    __shared__ BeamCand sset[2][SCAP];
    __shared__ float tw[2][4];
    __shared__ int scnt[2];
    // block-uniform result: true = out[0..K2) written from S
    auto fast = [&](unsigned ok, BeamCand* out, int L) -> bool {
        const int lane = tid & 63;
        const unsigned al = ok & live;
        float lm = -INFINITY;
#pragma unroll
        for (int u = 0; u < TOPK_VPT; ++u)
            if ((al >> u) & 1u) lm = fmaxf(lm, xv[u]);
        // K2 wave maxima of the lane maxima, each popped lane dropping out (below -inf)
        int c = score_key(lm), t = INT_MIN;
        for (int r = 0; r < K2; ++r) {
            t = wave_max_key(c);
            if (lane == __ffsll((long long)__ballot(c == t)) - 1) c = INT_MIN;
        }
        if (lane == 0) tw[L][tid >> 6] = score_of(t);
        if (tid == 0) scnt[L] = 0;
        __syncthreads();
        const float T = fmaxf(fmaxf(tw[L][0], tw[L][1]), fmaxf(tw[L][2], tw[L][3]));
        if (T == -INFINITY) return false;
        unsigned qm = 0;
#pragma unroll
        for (int u = 0; u < TOPK_VPT; ++u)
            if (((al >> u) & 1u) && xv[u] >= T) qm |= 1u << u;
        if (qm) {
            int bi = lo + tid;
            asm volatile("" : "+v"(bi));  // token ids not shared with (kept live for) the pops
            int k = atomicAdd(&scnt[L], __popc(qm));
#pragma unroll
            for (int u = 0; u < TOPK_VPT; ++u)
                if ((qm >> u) & 1u) {
                    if (k < SCAP) sset[L][k] = BeamCand{xv[u], bi + u * 256};
                    ++k;
                }
        }
        __syncthreads();
        const int n = scnt[L];
        if (n > SCAP) return false;
        if (n <= 64) {  // wave 0, one member per lane
            if (tid < 64) {
                const BeamCand e = sset[L][min(tid, n - 1)];
                const int rank = wave_rank(tid < n ? rank_key(e.s, e.i) : 0ull, n);
                if (tid < n && rank < K2) out[rank] = e;
            }
            return true;
        }
        for (int i = tid; i < n; i += 256) {
            const BeamCand e = sset[L][i];
            int rank = 0;
#pragma unroll 1
            for (int j = 0; j < n; ++j) {
                const BeamCand f = sset[L][j];
                rank += (f.s > e.s || (f.s == e.s && f.i < e.i)) ? 1 : 0;
            }
            if (rank < K2) out[rank] = e;
        }
        return true;
    };
    if (!FAST || !fast(okA, outA, 0)) pops(okA, outA);
    if (hi > P.tb) {
        if (!FAST || !fast(okB, outB, 1)) pops(okB, outB);
    }
    else if (tid < K2) outB[tid] = BeamCand{-INFINITY, INT_MAX};  // no timestamps in this slice
    __syncthreads();
    if (tid == 0) {
        SelPart r = wp[0];
        for (int i = 1; i < 4; ++i) {
            const SelPart& q = wp[i];
            lse_merge(r.m_all, r.s_all, q.m_all, q.s_all);
            lse_merge(r.m_ts, r.s_ts, q.m_ts, q.s_ts);
            ArgMax A = amax(ArgMax{r.v_all, r.i_all}, ArgMax{q.v_all, q.i_all});
            ArgMax X = amax(ArgMax{r.v_text, r.i_text}, ArgMax{q.v_text, q.i_text});
            ArgMax T = amax(ArgMax{r.v_ts, r.i_ts}, ArgMax{q.v_ts, q.i_ts});
            r.v_all = A.v; r.i_all = A.i; r.v_text = X.v; r.i_text = X.i; r.v_ts = T.v; r.i_ts = T.i;
        }
        parts[b * SEL_SPLIT + sl] = r;  // read by beam_update, a later launch
    }
}

// grid (rows, SEL_SPLIT), 256 threads: every slice of a row computes its partial
// and takes the row's arrival ticket (also slices that have nothing to do, so the
// finaliser knows every slice has read the step counter); the last one combines the
// slices in fixed order and picks the row's token (select_final_row).  With `bump`
// (greedy steps) the last row to be finalised advances the device step counter: by
// then every slice of every row has read it.  One launch instead of partial + final.
// MODE 0: greedy rows, 1: sampling rows (temperature > 0), 2: beam rows.  Each launch
// compiles only its own path: the greedy kernel carries neither the Gumbel keys nor the
// beam candidate lists (47 VGPRs, so it fits beside another lane's encoder workgroup).
template <int MODE>
// waves_per_eu(6): <= 80 VGPRs (the beam form needs 81 unbounded), so it fits beside an encoder GEMM workgroup
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void select_kernel(const float* __restrict__ logits, SelParams P,
                                                     int* __restrict__ pos_ptr, const unsigned* __restrict__ supmask,
                                                     const int* __restrict__ prompt, SelPart* __restrict__ parts,
                                                     SelState* __restrict__ st, int* __restrict__ cur_tok,
                                                     int* __restrict__ tokens, int max_tokens,
                                                     int* __restrict__ arrive, int* __restrict__ ticket, int bump,
                                                     BeamCand* __restrict__ cand) {
    const int step = pos_ptr[P.pos_row ? blockIdx.x : 0];
    if ((MODE == 2 || MODE == 3) && P.beam > 1) {
        const SelState s = st[blockIdx.x];
        if (sel_mode(P, step, s) == SEL_SAMPLE) {  // the same for every slice of the row
            // beam rows' sampling steps: statistics + candidates in one pass; nothing to
            // finalise here (beam_update picks), so no ticket
            if (step == row_plen(P, s) - 1 && blockIdx.x % P.beam != 0) return;  // only the prompt hypothesis expands
            beam_slice_body<MODE == 2>(logits, P, step, supmask, s, parts, cand);
            return;
        }
    }
    select_partial_body<MODE == 1>(logits, P, step, supmask, st, parts);
    __shared__ int last;
    __shared__ SelPart rp[SEL_SPLIT];
    const int b = blockIdx.x;
    if (threadIdx.x == 0) {
        __builtin_amdgcn_s_waitcnt(0);  // this slice's part stores are complete at device scope
        last = __hip_atomic_fetch_add(ticket + b, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == SEL_SPLIT - 1;
        if (last) __hip_atomic_store(ticket + b, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
    }
    __syncthreads();
    if (!last) return;
    // one lane per slice fetches it (device scope: written by other workgroups, maybe
    // on other XCDs); thread 0 combines them in fixed order
    if (threadIdx.x < SEL_SPLIT) rp[threadIdx.x] = load_part(parts + b * SEL_SPLIT + threadIdx.x);
    __syncthreads();
    if (threadIdx.x != 0) return;
    select_final_row(logits, P, step, prompt, rp, st, cur_tok, tokens, max_tokens);
    if (!bump) return;
    if (P.pos_row) {  // row refill: every slice of this row has read its own counter
        __builtin_amdgcn_s_waitcnt(0);
        __hip_atomic_store(pos_ptr + b, step + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    __builtin_amdgcn_s_waitcnt(0);
    if (__hip_atomic_fetch_add(arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1) {
        __hip_atomic_store(arrive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(pos_ptr, step + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---------------------------------------------------------------------------
// Beam search (restated CTranslate2 BeamSearch, see oracle/decode.py): per row the
// processed log-probs (rules + log-softmax, timestamp-mass rule) plus the row's
// cumulative score; per window the top 2*beam candidates over beam x vocab, the
// finished-hypothesis bookkeeping and the reorder of the surviving hypotheses.
// The KV cache is never copied: row r's key at position p lives in the slot of row
// anc[r][p] (written at step p); the reorder copies only anc / tokens / state.


// grid windows, 256 threads: merge the candidates, register finished hypotheses,
// pick the surviving beams and reorder their tokens / ancestry / state.
// KM: the largest beam the LDS arrays hold (5, the reference's beam_size: 24 KiB, so the
// workgroup fits beside another lane's 128-KiB encoder workgroup; 8: 45 KiB)
#ifdef OSW_STAMPS
// diagnostic build only (make EXTRA=-DOSW_STAMPS): phase times of the last beam_update launch
// whose workgroup 0 ran the whole update (staged in [16, 28), flag 31), read by
// osw_debug_stamps (never part of the product library).  OSW_STAMP_LAST closes a launch.
__device__ unsigned long long osw_stamps[32];
#define OSW_STAMP(i)                                                                        \
    do {                                                                                    \
        __builtin_amdgcn_sched_barrier(0);                                                  \
        unsigned long long t_;                                                              \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");          \
        __builtin_amdgcn_sched_barrier(0);                                                  \
        if (blockIdx.x == 0 && threadIdx.x == 0) osw_stamps[16 + (i)] = t_;                 \
    } while (0)
#define OSW_STAMP_FULL()                                                                    \
    do {                                                                                    \
        if (blockIdx.x == 0 && threadIdx.x == 0) osw_stamps[31] = 1;                        \
    } while (0)
#define OSW_STAMP_LAST(i)                                                                   \
    do {                                                                                    \
        OSW_STAMP(i);                                                                       \
        if (blockIdx.x == 0 && threadIdx.x == 0 && osw_stamps[31]) {                        \
            for (int j_ = 0; j_ <= (i); ++j_) osw_stamps[j_] = osw_stamps[16 + j_];         \
            osw_stamps[31] = 0;                                                             \
        }                                                                                   \
    } while (0)
#else
#define OSW_STAMP(i) \
    do {             \
    } while (0)
#define OSW_STAMP_FULL() \
    do {                 \
    } while (0)
#define OSW_STAMP_LAST(i) \
    do {                  \
    } while (0)
#endif

template <int KM>
__device__ __forceinline__ void beam_update_body(const SelParams& P, const int* __restrict__ pos_ptr,
                                                          SelState* __restrict__ st, const SelPart* __restrict__ parts,
                                                          const BeamCand* __restrict__ cand, int* __restrict__ seq,
                                                          int* __restrict__ anc, int ctx, BeamWin* __restrict__ bwin,
                                                          int* __restrict__ best_tok, int* __restrict__ cur_tok,
                                                          int max_tokens) {
    constexpr int MAXC = KM * BEAM_SLICES * 2 * KM;
    constexpr int CPT = (MAXC + 255) / 256;      // candidates per thread
    __shared__ BeamCand top[2 * KM];
    __shared__ ArgMax wtop[4 * 2 * KM];
    __shared__ int lseq[KM][448];
    __shared__ int lanc[KM][448];
    __shared__ SelState lst[KM];
    __shared__ int ch_src[KM], ch_tok[KM], fin, best_src, best_extra, improved;
    __shared__ float ch_score[KM];
    OSW_STAMP(0);
    const int w = blockIdx.x, tid = threadIdx.x, K = P.beam, K2 = 2 * K;
    const int r0 = w * K;
    const int step = pos_ptr[P.pos_row ? r0 : 0];
    const SelState s0 = st[r0];
    const int nc = K * BEAM_SLICES * K2;
    // Loads are issued before any is used, in two round trips: with the window's state (before
    // its mode is known; wasted only by a window that is not sampling) both candidate lists of
    // every (row, slice) (the row's timestamp rule, known only once its 16 slice statistics
    // are combined, picks one), the slice statistics and the rows' states; then the token
    // histories and ancestry, whose extents need the state.  Clamped addresses.
    // (flat candidate index i = (k * BEAM_SLICES + slice) * K2 + e: divisions by the runtime
    // K2 through a float reciprocal, exact with the correction for i < 2^22)
    const float rk2 = 1.f / (float)K2;
    auto div_k2 = [&](int x) {
        int q = (int)((float)x * rk2);
        q -= q * K2 > x ? 1 : 0;
        q += (q + 1) * K2 <= x ? 1 : 0;
        return q;
    };
    BeamCand ca[CPT], cb[CPT];
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
        const int i = min(tid + 256 * j, nc - 1), qe = div_k2(i);  // qe = k * BEAM_SLICES + slice
        const BeamCand* src = cand + ((int64_t)(r0 * BEAM_SLICES + qe) * 2) * MAXK2 + (i - qe * K2);
        ca[j] = src[0];
        cb[j] = src[MAXK2];
    }
    SelPart mp{};
    if (tid < K * SEL_SPLIT) mp = parts[(int64_t)r0 * SEL_SPLIT + tid];
    SelState ms{};
    if (tid < K) ms = st[r0 + tid];
    BeamWin bw{};  // the window's finished-hypothesis record and token budget (thread 0)
    int budget = 0;
    if (tid == 0) {
        bw = bwin[w];
        budget = P.budget ? P.budget[r0] : 0;
    }
    if (sel_mode(P, step, s0) != SEL_SAMPLE) return;
    OSW_STAMP(1);
    const int n = s0.n_sampled;  // identical for every row of the window
    const int plen = row_plen(P, s0);
    const bool first = step == plen - 1;  // only the prompt hypothesis expands
    // token histories and ancestry: row k, positions tid and tid + 256 (both < 448)
    int hv[KM][2], av[KM][2];
#pragma unroll
    for (int k = 0; k < KM; ++k)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int kk = min(k, K - 1), jj = tid + 256 * h;
            hv[k][h] = seq[(int64_t)(r0 + kk) * max_tokens + min(jj, min(max(n, 1), max_tokens) - 1)];
            av[k][h] = anc[(int64_t)(r0 + kk) * ctx + min(jj, max(step, 1) - 1)];
        }
    if (tid < K) lst[tid] = ms;
#pragma unroll
    for (int k = 0; k < KM; ++k) {
        if (k >= K) break;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int jj = tid + 256 * h;
            if (jj < n) lseq[k][jj] = hv[k][h];
            if (jj < step) lanc[k][jj] = av[k][h];
        }
    }
    // per row: lse over the allowed tokens, over the allowed timestamps, and the
    // timestamp-mass rule.  Lane k * SEL_SPLIT + slice holds slice statistics of row k; a
    // butterfly merges the row's 16 (lse_merge and amax commute, so every lane of the group
    // ends with the same statistics)
    static_assert(SEL_SPLIT == 16, "one 16-lane DPP row per beam row");
    __shared__ float rlse[KM], rsum[KM];
    __shared__ int rts[KM];
    {
        float m_all = mp.m_all, s_all = mp.s_all, m_ts = mp.m_ts, s_ts = mp.s_ts;
        ArgMax X{mp.v_text, mp.i_text};
        auto bfly = [&](auto o) {
            constexpr int O = decltype(o)::value;
            const float ma = xor_lane<O>(m_all), sa = xor_lane<O>(s_all);
            const float mt = xor_lane<O>(m_ts), stt = xor_lane<O>(s_ts);
            const ArgMax x{xor_lane<O>(X.v), xor_lane<O>(X.i)};
            lse_merge(m_all, s_all, ma, sa);
            lse_merge(m_ts, s_ts, mt, stt);
            X = amax(X, x);
        };
        bfly(IC<1>{}), bfly(IC<2>{}), bfly(IC<4>{}), bfly(IC<8>{});
        if (tid < K * SEL_SPLIT && (tid & (SEL_SPLIT - 1)) == 0) {
            const int k = tid / SEL_SPLIT;
            const float lse_all = m_all + logf(s_all);
            const float lse_ts = m_ts == -INFINITY ? -INFINITY : m_ts + logf(s_ts);
            const bool ts_wins = P.with_ts && lse_ts - lse_all > X.v - lse_all;
            rlse[k] = ts_wins ? lse_ts : lse_all;
            rts[k] = ts_wins;
        }
        if (tid < K) rsum[tid] = ms.sum_lp;
    }
    __syncthreads();
    OSW_STAMP(2);
    OSW_STAMP(3);
    {
        // the top K2 candidates by (score desc, flat id asc), NaN scores and INT_MAX ids
        // excluded, {-inf, INT_MAX} past the last valid one.  Each wave pops its own top K2
        // (wave max of the lanes' best scores, a ballot for ties; flat ids are unique, so
        // one lane owns each pop and shifts its sorted list), then wave 0 ranks the 4*K2
        // survivors: the global top K2 lie among them, so this is the list (and order) of
        // K2 block-wide pops, with one barrier instead of 2*K2.
        const int lane = tid & 63, wv = tid >> 6;
        // candidate (row k, slice, j): list B if the row's timestamps win, else list A; score =
        // sum_lp + (x - lse) as the per-row log-prob + cumulative score of the reference
        // ck: the score as an int ordered like the float (-0 as +0; dead: INT_MIN), so wave
        // maxima are integer DPP maxima and equal keys are equal scores
        // (an involution: the score is read back from the key)
        int cx[CPT], ck[CPT];
#pragma unroll
        for (int j = 0; j < CPT; ++j) {
            const int i = tid + 256 * j;
            cx[j] = INT_MAX;
            ck[j] = INT_MIN;
            if (i < nc) {
                const int k = div_k2(i) / BEAM_SLICES;
                const BeamCand c = rts[k] ? cb[j] : ca[j];
                const float v = rsum[k] + (c.s - rlse[k]);
                if (c.i != INT_MAX && !(first && k != 0) && !(v != v)) {
                    cx[j] = k * P.V + c.i;
                    ck[j] = score_key(v);
                }
            }
        }
        // this lane's candidates best first (amax order)
#pragma unroll
        for (int a = 1; a < CPT; ++a)
#pragma unroll
            for (int b = a; b > 0; --b) {
                const bool sw = ck[b] > ck[b - 1] || (ck[b] == ck[b - 1] && cx[b] < cx[b - 1]);
                const int ti = cx[b], tk = ck[b];
                cx[b] = sw ? cx[b - 1] : ti;
                ck[b] = sw ? ck[b - 1] : tk;
                cx[b - 1] = sw ? ti : cx[b - 1];
                ck[b - 1] = sw ? tk : ck[b - 1];
            }
        for (int r = 0; r < K2; ++r) {
            const int m = wave_max_key(ck[0]);
            const unsigned long long tie = __ballot(ck[0] == m);
            int owner = __ffsll((long long)tie) - 1;
            if (__popcll(tie) > 1) {  // equal scores: the smallest flat id
                int im = ck[0] == m ? cx[0] : INT_MAX;
                im = min(im, xor_lane<32>(im));
                im = min(im, xor_lane<16>(im));
                im = min(im, xor_lane<8>(im));
                im = min(im, xor_lane<4>(im));
                im = min(im, xor_lane<2>(im));
                im = min(im, xor_lane<1>(im));
                owner = __ffsll((long long)__ballot(ck[0] == m && cx[0] == im)) - 1;
            }
            if (lane == 0)
                wtop[wv * K2 + r] = ArgMax{score_of(m),
                                           __builtin_amdgcn_readlane(cx[0], owner)};
            if (lane == owner) {
#pragma unroll
                for (int j = 0; j + 1 < CPT; ++j) {
                    cx[j] = cx[j + 1];
                    ck[j] = ck[j + 1];
                }
                cx[CPT - 1] = INT_MAX;
                ck[CPT - 1] = INT_MIN;
            }
        }
        OSW_STAMP(4);
        __syncthreads();
        OSW_STAMP(5);
        if (wv == 0) {
            const int S = 4 * K2;  // <= 64 (K2 <= 2 * KM <= 16)
            const ArgMax e = lane < S ? wtop[lane] : ArgMax{-INFINITY, INT_MAX};
            const bool valid = lane < S && e.i != INT_MAX;
            const int rank = wave_rank(valid ? rank_key(e.v, e.i) : 0ull, S);
            const int nvalid = __popcll(__ballot(valid));
            if (valid && rank < K2) top[rank] = BeamCand{e.v, e.i};
            if (lane < K2 && lane >= nvalid) top[lane] = BeamCand{-INFINITY, INT_MAX};
        }
        __syncthreads();
    }
    OSW_STAMP(6);
    if (tid < 64) {
        // wave 0: lane j decodes top[j] (token, and whether it is <|endoftext|>); lane 0
        // walks the K hypotheses in order with the values read back from the lanes
        const BeamCand cj = top[min(tid, K2 - 1)];
        const int srcj = cj.i == INT_MAX ? 0 : cj.i / P.V;  // source row
        const int tokj = cj.i == INT_MAX ? P.eot : cj.i - srcj * P.V;
        const unsigned cont = (unsigned)__ballot(tid < K2 && tokj != P.eot);  // continuations
        float cs[KM];
        int ct[KM];
#pragma unroll
        for (int k = 0; k < KM; ++k) {
            cs[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cj.s), k));
            ct[k] = __builtin_amdgcn_readlane(tokj, k);
        }
        if (tid == 0) {
            // the last step: max_length, or (length control) the window's token budget
            const bool is_last = plen + n + 1 >= P.max_length || (budget > 0 && n + 1 >= budget);
            int sec = K;
            bool top_fin = false;
            improved = 0;
#pragma unroll
            for (int k = 0; k < KM; ++k) {
                if (k >= K) break;
                const int tok = ct[k];
                int nb = k;
                if (tok == P.eot || is_last) {
                    if (k == 0) top_fin = true;
                    const int len = n + (tok == P.eot ? 0 : 1);
                    const float norm = len == 0 ? (P.length_penalty != 0.f ? -INFINITY : cs[k])
                                                : cs[k] / powf((float)len, P.length_penalty);
                    bw.n_hyp += 1;
                    if (bw.n_hyp == 1 || norm > bw.best_norm) {
                        bw.best_norm = norm;
                        bw.best_raw = cs[k];
                        bw.best_len = min(len, max_tokens);
                        best_src = __builtin_amdgcn_readlane(srcj, k);
                        best_extra = tok == P.eot ? -1 : tok;
                        improved = 1;
                    }
                    // the next continuation at or after position sec replaces it
                    const unsigned rest = cont & ~((1u << sec) - 1u);
                    if (rest) {
                        nb = __ffs(rest) - 1;
                        sec = nb + 1;
                    }
                }
                // row k continues hypothesis nb
                ch_src[k] = __builtin_amdgcn_readlane(srcj, nb);
                ch_tok[k] = __builtin_amdgcn_readlane(tokj, nb);
                ch_score[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cj.s), nb));
            }
            fin = is_last || (top_fin && bw.n_hyp >= P.num_hyp) || bw.n_hyp >= P.max_cand;
            bw.done = fin;
            bwin[w] = bw;
        }
    }
    __syncthreads();
    OSW_STAMP(7);
    if (improved) {
        int* dst = best_tok + (int64_t)w * max_tokens;
        for (int j = tid; j < n && j < max_tokens; j += 256) dst[j] = lseq[best_src][j];
        if (tid == 0 && best_extra >= 0 && n < max_tokens) dst[n] = best_extra;
    }
    if (fin) {
        if (tid < K) {
            SelState s2 = lst[tid];
            s2.done = 1;
            st[r0 + tid] = s2;
            cur_tok[r0 + tid] = P.eot;
        }
        return;
    }
    // row k continues hypothesis (ch_src, ch_tok, ch_score)[k]: its source row's history
    // (positions tid and tid + 256, both < 448) and ancestry, then the state (thread k)
    int qk[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) qk[k] = ch_src[min(k, K - 1)];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
        if (k >= K) break;
        int* sq = seq + (int64_t)(r0 + k) * max_tokens;
        int* an = anc + (int64_t)(r0 + k) * ctx;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int j = tid + 256 * h;
            if (j < n && j < max_tokens) sq[j] = lseq[qk[k]][j];
            if (j <= step && j < ctx) an[j] = j < step ? lanc[qk[k]][j] : r0 + qk[k];
        }
    }
    if (tid < K) {
        const int q = ch_src[tid], tok = ch_tok[tid];
        if (n < max_tokens) seq[(int64_t)(r0 + tid) * max_tokens + n] = tok;
        SelState s2 = lst[q];
        s2.n_sampled = n + 1;
        s2.penult = s2.last;
        s2.last = tok;
        if (tok >= P.tb) s2.last_ts = tok;
        s2.sum_lp = ch_score[tid];
        st[r0 + tid] = s2;
        cur_tok[r0 + tid] = tok;
    }
    OSW_STAMP(8);
    OSW_STAMP_FULL();
}

// grid windows: the per-window merge / finish / reorder, then an arrival count over
// the windows; the last one advances the device step counter (every window read it
// at its start), so beam steps need no separate bump launch.
template <int KM>
__global__ __launch_bounds__(256) void beam_update_kernel(SelParams P, int* __restrict__ pos_ptr,
                                                          SelState* __restrict__ st, const SelPart* __restrict__ parts,
                                                          const BeamCand* __restrict__ cand, int* __restrict__ seq,
                                                          int* __restrict__ anc, int ctx, BeamWin* __restrict__ bwin,
                                                          int* __restrict__ best_tok, int* __restrict__ cur_tok,
                                                          int max_tokens, int* __restrict__ arrive) {
    const int step = pos_ptr[P.pos_row ? blockIdx.x * P.beam : 0];
    beam_update_body<KM>(P, pos_ptr, st, parts, cand, seq, anc, ctx, bwin, best_tok, cur_tok, max_tokens);
    __syncthreads();
    OSW_STAMP_LAST(9);
    if (P.pos_row) {  // a session: this window's rows advance their own counters
        if (threadIdx.x < P.beam) pos_ptr[blockIdx.x * P.beam + threadIdx.x] = step + 1;
        return;
    }
    if (threadIdx.x != 0) return;
    __builtin_amdgcn_s_waitcnt(0);
    if (__hip_atomic_fetch_add(arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1) {
        __hip_atomic_store(arrive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(pos_ptr, step + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Row refill (osw.hip decode_refill): reset the decoder rows of newly admitted windows.
// pack[i] = {row, token budget, prompt[0 .. P)}; one workgroup per admitted window.
__global__ __launch_bounds__(64) void refill_rows_kernel(const int* __restrict__ pack, int P, int* __restrict__ prompt,
                                                         int* __restrict__ budget, int* __restrict__ cur_tok,
                                                         int* __restrict__ pos, SelState* __restrict__ st) {
    const int* e = pack + (int64_t)blockIdx.x * (2 + P);
    const int row = e[0];
    for (int j = threadIdx.x; j < P; j += blockDim.x) prompt[(int64_t)row * P + j] = e[2 + j];
    if (threadIdx.x == 0) {
        if (budget) budget[row] = e[1];
        cur_tok[row] = e[2];
        pos[row] = 0;
        st[row] = SelState{};
    }
}

// Decode sessions (osw.hip, osw_session_*): reset the `group` rows of each admitted window
// slot.  pack[i] = {slot, plen, budget, prompt[0 .. plen)} with stride `ps`; grid (windows,
// group), 64 threads.  Beam rows (anc != nullptr) also get an identity ancestry and the
// window's hypothesis bookkeeping a fresh start.
__global__ __launch_bounds__(64) void session_rows_kernel(const int* __restrict__ pack, int ps, int group,
                                                          int pstride, int ctx, int* __restrict__ prompt,
                                                          int* __restrict__ budget, int* __restrict__ cur_tok,
                                                          int* __restrict__ pos, SelState* __restrict__ st,
                                                          int* __restrict__ anc, BeamWin* __restrict__ bwin) {
    const int* e = pack + (int64_t)blockIdx.x * ps;
    const int slot = e[0], plen = e[1];
    const int row = slot * group + blockIdx.y;
    for (int j = threadIdx.x; j < plen; j += blockDim.x) prompt[(int64_t)row * pstride + j] = e[3 + j];
    if (anc)
        for (int p = threadIdx.x; p < ctx; p += blockDim.x) anc[(int64_t)row * ctx + p] = row;
    if (threadIdx.x == 0) {
        budget[row] = e[2];
        cur_tok[row] = e[3];
        pos[row] = 0;
        SelState s{};
        s.plen = plen;
        st[row] = s;
        if (bwin && blockIdx.y == 0) bwin[slot] = BeamWin{};
    }
}

__global__ void count_done_kernel(const SelState* st, int B, int* out) {
    int c = 0;
    for (int i = threadIdx.x; i < B; i += blockDim.x) c += st[i].done;
    c = (int)wave_sum((float)c);
    if (threadIdx.x == 0) *out = c;
}

}  // namespace

void launch_refill_rows(const int* pack, int k, int P, int* prompt, int* budget, int* cur_tok, int* pos, SelState* st,
                        hipStream_t s) {
    refill_rows_kernel<<<k, 64, 0, s>>>(pack, P, prompt, budget, cur_tok, pos, st);
}

int sel_parts_bytes() { return (int)sizeof(SelPart) * SEL_SPLIT; }
int sel_fused_parts_bytes(int V) { return (int)sizeof(SelPart) * ((V + 63) / 64); }
int beam_cand_bytes(int) { return (int)sizeof(BeamCand) * BEAM_SLICES * 2 * MAXK2; }

void launch_dec_self_attn(const float* part, int ks, const float* bias, h16* kc, h16* vc, const int* pos, int B,
                          int H, int ctx, h16* out, int64_t lo_off, const int* anc, int group, const SelState* st,
                          hipStream_t s, int pos_row) {
    // V issued with K (VPRE, 139 VGPRs) only for a few rows: batch-1 p50 114.3 / 114.8 ->
    // 113.6 / 113.4 ms greedy, 152.2 / 153.5 -> 151.6 / 151.4 ms beam 5; at 64 rows its 3
    // waves per SIMD lose to the 7 of the 66-VGPR form (16.9 -> 20.8 us per launch, beam rows
    // 49.0 -> 66.6 us; gpurun_out/r03_ae).  OSW_SELF_VPRE=0 / 1: never / always.
    static const int vpre_env = [] {
        const char* e = std::getenv("OSW_SELF_VPRE");
        return e ? (e[0] == '1' ? 1 : 0) : -1;
    }();
    static const int vpre_rows = [] {  // OSW_SELF_VPRE_ROWS=n: the row limit of the default
        const char* e = std::getenv("OSW_SELF_VPRE_ROWS");
        return e ? atoi(e) : 8;
    }();
    const bool vlate = vpre_env < 0 ? B > vpre_rows : vpre_env == 0;
    // OSW_SELF_KALL (A/B switch; bit 1: the V-late form, bit 2: the VPRE form): both 256-key
    // blocks' K (and V) pieces issued before any is used (attend_one KALL; same bits)
    static const int kall = [] {
        const char* e = std::getenv("OSW_SELF_KALL");
        return e ? atoi(e) : 0;
    }();
    if (anc) {  // ctx <= 448 (osw.hip checks the context at decode)
        if (vlate)
            dec_self_attn_kernel<true, false><<<H * B, 256, 0, s>>>(part, ks, bias, kc, vc, pos, H, B, ctx, out, lo_off,
                                                                    anc, group, st, pos_row);
        else
            dec_self_attn_kernel<true, true><<<H * B, 256, 0, s>>>(part, ks, bias, kc, vc, pos, H, B, ctx, out, lo_off,
                                                                   anc, group, st, pos_row);
    } else if (vlate) {
        if (kall & 1)
            dec_self_attn_kernel<false, false, true><<<H * B, 256, 0, s>>>(part, ks, bias, kc, vc, pos, H, B, ctx, out,
                                                                           lo_off, nullptr, 1, st, pos_row);
        else
            dec_self_attn_kernel<false, false><<<H * B, 256, 0, s>>>(part, ks, bias, kc, vc, pos, H, B, ctx, out, lo_off,
                                                                     nullptr, 1, st, pos_row);
    } else {
        if (kall & 2)
            dec_self_attn_kernel<false, true, true><<<H * B, 256, 0, s>>>(part, ks, bias, kc, vc, pos, H, B, ctx, out,
                                                                          lo_off, nullptr, 1, st, pos_row);
        else
            dec_self_attn_kernel<false, true><<<H * B, 256, 0, s>>>(part, ks, bias, kc, vc, pos, H, B, ctx, out, lo_off,
                                                                    nullptr, 1, st, pos_row);
    }
}

void launch_dec_cross_attn(const float* part, int ks, const float* bias, const h16* xk, const h16* xv, int B, int H,
                           int T, int beam, h16* out, int64_t lo_off, float* ws, int* ticket, const SelState* st,
                           hipStream_t s) {
    static const bool legacy = std::getenv("OSW_XATTN_LEGACY") != nullptr;  // A/B switch: one workgroup per (row, head)
    if (legacy || !ws) {
        dec_cross_attn_kernel<<<H * B, 256, 0, s>>>(part, ks, bias, xk, xv, H, B, T, beam, out, lo_off);
        return;
    }
    const int W = B / beam;
    const unsigned grid = (unsigned)(((W * H + 7) / 8) * 8 * XCH);
    static const bool valu_beam = std::getenv("OSW_XATTN_VALU") != nullptr;  // A/B switch
    if (beam > 1 && !valu_beam && ks <= 8) {
        static const bool kdirect = std::getenv("OSW_XATTN_KDIRECT") != nullptr;  // A/B switch
        if (kdirect) {
            if (beam <= 5) dec_xattn_mfma_kernel<5, false><<<grid, 256, 0, s>>>(part, ks, bias, xk, xv, H, W, T, beam, ws, ticket, out, lo_off, st);
            else dec_xattn_mfma_kernel<8, false><<<grid, 256, 0, s>>>(part, ks, bias, xk, xv, H, W, T, beam, ws, ticket, out, lo_off, st);
        } else {
            if (beam <= 5) dec_xattn_mfma_kernel<5><<<grid, 256, 0, s>>>(part, ks, bias, xk, xv, H, W, T, beam, ws, ticket, out, lo_off, st);
            else dec_xattn_mfma_kernel<8><<<grid, 256, 0, s>>>(part, ks, bias, xk, xv, H, W, T, beam, ws, ticket, out, lo_off, st);
        }
        return;
    }
    switch (beam) {
        case 1: dec_xattn_chunk_kernel<1><<<grid, 256, 0, s>>>(part, ks, bias, xk, xv, H, W, T, beam, ws, ticket, out, lo_off, st); break;
        case 2: dec_xattn_chunk_kernel<2><<<grid, 256, 0, s>>>(part, ks, bias, xk, xv, H, W, T, beam, ws, ticket, out, lo_off, st); break;
        case 3:
        case 4: dec_xattn_chunk_kernel<4><<<grid, 256, 0, s>>>(part, ks, bias, xk, xv, H, W, T, beam, ws, ticket, out, lo_off, st); break;
        case 5: dec_xattn_chunk_kernel<5><<<grid, 256, 0, s>>>(part, ks, bias, xk, xv, H, W, T, beam, ws, ticket, out, lo_off, st); break;
        default: dec_xattn_chunk_kernel<8><<<grid, 256, 0, s>>>(part, ks, bias, xk, xv, H, W, T, beam, ws, ticket, out, lo_off, st); break;
    }
}

void launch_dec_resid_ln(const float* part, int ks, int B, int D, const float* bias, float* x, const float* g,
                         const float* be, h16* y, int64_t lo_off, const h16* tok_emb, const float* pos_emb,
                         const int* tok, const int* pos, int ctx, int V, hipStream_t s, int pos_row) {
    ResLnArgs A{part, ks, (int64_t)B * D, bias, x, x, g, be, tok_emb, pos_emb, tok, pos, ctx, D, V, pos_row};
    dec_resid_ln_kernel<<<B, 256, 0, s>>>(A, y, lo_off);
}

void launch_dec_reduce_gelu(const float* part, int ks, int B, int N, const float* bias, h16* y, int64_t lo_off,
                            hipStream_t s) {
    const int64_t total = (int64_t)B * N;
    dec_reduce_gelu_kernel<<<(unsigned)std::min<int64_t>((total + 255) / 256, 1024), 256, 0, s>>>(part, ks, total, N,
                                                                                                 bias, y, lo_off);
}

void launch_select(const float* logits, int rows, int* pos, const SelParams& P, const int* prompt,
                   const unsigned* supmask, SelState* st, int* cur_tok, int* tokens, int max_tokens, void* sel_parts,
                   int* arrive, bool bump, void* cand, hipStream_t s) {
    // arrive[0]: rows finalised this step; arrive[1 + row]: the row's slice tickets; cand:
    // the beam rows' candidate lists (beam_slice_body)
    const dim3 grid(rows, SEL_SPLIT);
    // OSW_BEAM_POPS=1 (A/B switch): the beam candidate lists by K2 block-wide pops everywhere
    static const bool pops_only = std::getenv("OSW_BEAM_POPS") != nullptr;
    if (P.beam > 1 && pops_only)
        select_kernel<3><<<grid, 256, 0, s>>>(logits, P, pos, supmask, prompt, (SelPart*)sel_parts, st, cur_tok, tokens,
                                               max_tokens, arrive, arrive + 1, bump ? 1 : 0, (BeamCand*)cand);
    else if (P.beam > 1)
        select_kernel<2><<<grid, 256, 0, s>>>(logits, P, pos, supmask, prompt, (SelPart*)sel_parts, st, cur_tok, tokens,
                                               max_tokens, arrive, arrive + 1, bump ? 1 : 0, (BeamCand*)cand);
    else if (P.inv_temp > 0.f)
        select_kernel<1><<<grid, 256, 0, s>>>(logits, P, pos, supmask, prompt, (SelPart*)sel_parts, st, cur_tok, tokens,
                                               max_tokens, arrive, arrive + 1, bump ? 1 : 0, (BeamCand*)cand);
    else
        select_kernel<0><<<grid, 256, 0, s>>>(logits, P, pos, supmask, prompt, (SelPart*)sel_parts, st, cur_tok, tokens,
                                               max_tokens, arrive, arrive + 1, bump ? 1 : 0, (BeamCand*)cand);
}

void launch_beam(const float* logits, int windows, int* pos, const SelParams& P, const unsigned* supmask,
                 SelState* st, const void* sel_parts, void* cand, int* seq, int* anc, int ctx, BeamWin* bw,
                 int* best_tok, int* cur_tok, int max_tokens, int* arrive, hipStream_t s) {
    if (P.beam <= 5)
        beam_update_kernel<5><<<windows, 256, 0, s>>>(P, pos, st, (const SelPart*)sel_parts, (const BeamCand*)cand, seq,
                                                      anc, ctx, bw, best_tok, cur_tok, max_tokens, arrive);
    else
        beam_update_kernel<MAX_BEAM><<<windows, 256, 0, s>>>(P, pos, st, (const SelPart*)sel_parts,
                                                             (const BeamCand*)cand, seq, anc, ctx, bw, best_tok, cur_tok,
                                                             max_tokens, arrive);
}

void launch_session_rows(const int* pack, int k, int ps, int group, int pstride, int ctx, int* prompt, int* budget,
                         int* cur_tok, int* pos, SelState* st, int* anc, BeamWin* bwin, hipStream_t s) {
    session_rows_kernel<<<dim3(k, group), 64, 0, s>>>(pack, ps, group, pstride, ctx, prompt, budget, cur_tok, pos, st,
                                                      anc, bwin);
}

void launch_count_done(const SelState* st, int rows, int* out, hipStream_t s) {
    count_done_kernel<<<1, 64, 0, s>>>(st, rows, out);
}


}  // namespace osw

#ifdef OSW_STAMPS
extern "C" int osw_debug_stamps(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(osw::osw_stamps), sizeof(unsigned long long) * 32, 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
