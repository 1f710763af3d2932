// Decoder self-attention of one (row, head), shared by the standalone kernel
// (decode.hip, dec_self_attn_kernel) and the batch-1 qkv GEMM's last-arriver tail
// (gemm.hip, TAIL_ATTN): the same functions, so both give the same bits.
// Included inside the anonymous namespace of each translation unit, after HD (= 64).

// a split-K slab value; DEV: written by another workgroup of the same launch (maybe on
// another XCD), so a device-scope load
template <bool DEV>
__device__ __forceinline__ float ldslab(const float* p) {
    if constexpr (DEV) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return *p;
}

__device__ __forceinline__ float block_reduce_max(float v, float* red) {
    v = wave_max(v);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) red[w] = v;
    __syncthreads();
    float r = red[0];
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) r = fmaxf(r, red[i]);
    return r;
}
__device__ __forceinline__ float block_reduce_sum(float v, float* red) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) red[w] = v;
    __syncthreads();
    float r = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) r += red[i];
    return r;
}

template <bool NT>
__device__ __forceinline__ h16x8 ld8(const h16* p) {
    if constexpr (NT) return __builtin_nontemporal_load((const h16x8*)p);
    return *(const h16x8*)p;
}

// Attention of one query row over n_keys rows of K/V ([n][64] fp16, contiguous);
// K/V loads are nontemporal (the self-K/V caches of a step exceed the MALL): 18.7 -> 17.1 us.
// 256 threads.  Scores live in LDS (n_keys <= MAXK).  Loads are issued in groups
// (8 K pieces = 256 keys, 8 V pieces = 256 keys per lane) before the FMAs that use
// them, so a 448-key cache costs two HBM round trips per pass (the former 128-key K
// tiles and one-piece V tail loop cost up to 4 and 8).  Thread t touches the keys
// (t >> 3) + 32 i (i = 0, 1, ...) in both passes.
//
// GATHER (beam search): key p of this row lives in the cache slot of the row that
// wrote position p of this hypothesis' history: K + soff[p] * slot_stride, where
// soff[p] = anc[p] - self (0 for the newest key, always this row's own), staged in LDS by
// the caller before its slab reduction's barrier, so the ancestry costs no round trip of
// its own.
// VPRE (the self-attention, MAXK = 448): each 256-key block's V pieces are issued with its K
// pieces, so the P·V pass finds them landed (one HBM round trip per block instead of two);
// the V pieces stay in registers across the softmax reductions.
// KALL (MAXK <= 512): both 256-key blocks' K pieces (and V pieces) are issued before any is
// used, so a 448-key cache costs one round trip per pass instead of two; the FMAs run in the
// same order, so the results are the same bits.
template <int MAXK, bool GATHER = false, bool NT = !GATHER, bool VPRE = false, bool KALL = false>
__device__ void attend_one(const h16* __restrict__ q16, const h16* __restrict__ K, const h16* __restrict__ V,
                           int n_keys, h16* __restrict__ out, int64_t lo_off, const int* soff = nullptr,
                           int64_t slot_stride = 0) {
    __shared__ float qs[HD];
    __shared__ float sc[MAXK];
    __shared__ float red[8];
    __shared__ f32x4 part[32][17];  // [key group][8 d-chunks x 2 float4]
    const int tid = threadIdx.x;
    if (tid < HD) qs[tid] = (float)q16[tid] * 0.125f;  // 1/sqrt(64), exact in fp32
    __syncthreads();
    auto krow = [&](const h16* base, int key) -> const h16* {
        // (32-bit element offsets: R rows x H x ctx x 64 < 2^31 at <= 1024 windows x 5 beams)
        if constexpr (GATHER) return base + (soff[key] * (int)slot_stride + key * HD);
        return base + (int64_t)key * HD;
    };
    constexpr int NBLK = (MAXK + 255) / 256;
    // scores: 8 lanes per key row (lane c holds dims 8c..8c+7), so one wave-instruction
    // reads 8 consecutive K rows = 1 KiB contiguous; 4 such loads in flight per lane;
    // the 8-lane partial dots are combined with 3 xor-shuffles.
    const int kg = tid >> 3, c8 = tid & 7;
    float q[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = qs[8 * c8 + i];
    float mx = -INFINITY;
    h16x8 vpre[VPRE ? NBLK : 1][8];
    static_assert(!KALL || NBLK <= 2, "KALL holds at most two blocks of pieces");
    auto kdots = [&](const h16x8 (&kv)[8], int base) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            float d = 0.f;
#pragma unroll
            for (int i = 0; i < 8; ++i) d = fmaf((float)kv[u][i], q[i], d);
            d += xor_lane<1>(d);
            d += xor_lane<2>(d);
            d += xor_lane<4>(d);
            const int key = base + u * 32 + kg;
            if (key < n_keys) {
                if (c8 == 0) sc[key] = d;
                mx = fmaxf(mx, d);
            }
        }
    };
    if constexpr (KALL) {
        h16x8 kv[NBLK][8];
#pragma unroll
        for (int blk = 0; blk < NBLK; ++blk) {
            const int base = blk * 256;
            if (base >= n_keys) break;
#pragma unroll
            for (int u = 0; u < 8; ++u) kv[blk][u] = ld8<NT>(krow(K, min(base + u * 32 + kg, n_keys - 1)) + 8 * c8);
            if constexpr (VPRE) {
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    vpre[blk][u] = ld8<NT>(krow(V, min(base + u * 32 + kg, n_keys - 1)) + 8 * c8);
            }
        }
#pragma unroll
        for (int blk = 0; blk < NBLK; ++blk) {
            if (blk * 256 >= n_keys) break;
            kdots(kv[blk], blk * 256);
        }
    } else {
    // 256 keys (8 loads per lane) per round trip: at most 2 for 448 keys
#pragma unroll
    for (int blk = 0; blk < NBLK; ++blk) {
        const int base = blk * 256;
        if (base >= n_keys) break;
        h16x8 kv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int key = min(base + u * 32 + kg, n_keys - 1);
            kv[u] = ld8<NT>(krow(K, key) + 8 * c8);
        }
        if constexpr (VPRE) {
#pragma unroll
            for (int u = 0; u < 8; ++u) vpre[blk][u] = ld8<NT>(krow(V, min(base + u * 32 + kg, n_keys - 1)) + 8 * c8);
        }
        kdots(kv, base);
    }
    }
    mx = block_reduce_max(mx, red);
    float sum = 0.f;
    for (int j = tid; j < n_keys; j += 256) {
        const float p = __expf(sc[j] - mx);
        sc[j] = p;
        sum += p;
    }
    sum = block_reduce_sum(sum, red);  // includes __syncthreads: sc visible
    // PV: thread -> (key group kg, d chunk c8), keys j = kg + 32 i; one wave-instruction
    // reads 8 consecutive V rows = 1 KiB contiguous
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // KALL without VPRE: every block's V pieces issued before the first block's FMAs
    h16x8 vall[KALL && !VPRE ? NBLK : 1][8];
    if constexpr (KALL && !VPRE) {
#pragma unroll
        for (int blk = 0; blk < NBLK; ++blk) {
            const int j = kg + blk * 256;
            if (blk * 256 >= n_keys) break;
#pragma unroll
            for (int u = 0; u < 8; ++u) vall[blk][u] = ld8<NT>(krow(V, min(j + 32 * u, n_keys - 1)) + 8 * c8);
        }
    }
    // 8 V pieces per lane per round trip (keys past the end: clamped address, p = 0, so
    // the lane's keys are still accumulated in increasing order with nothing added)
#pragma unroll
    for (int blk = 0; blk < NBLK; ++blk) {
        const int j = kg + blk * 256;
        if (j >= n_keys) break;
        h16x8 v[8];
        float p[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if constexpr (VPRE) v[u] = vpre[blk][u];
            else if constexpr (KALL) v[u] = vall[blk][u];
            else v[u] = ld8<NT>(krow(V, min(j + 32 * u, n_keys - 1)) + 8 * c8);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) p[u] = j + 32 * u < n_keys ? sc[j + 32 * u] : 0.f;
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[e] = fmaf(p[u], (float)v[u][e], acc[e]);
    }
    part[kg][2 * c8] = f32x4{acc[0], acc[1], acc[2], acc[3]};
    part[kg][2 * c8 + 1] = f32x4{acc[4], acc[5], acc[6], acc[7]};
    __syncthreads();
    if (tid < HD) {
        const int cc = tid >> 3, e = tid & 7;
        float r = 0.f;
        for (int k = 0; k < 32; ++k) r += part[k][2 * cc + (e >> 2)][e & 3];
        split_h16(r / sum, out, out + lo_off, tid);  // hi/lo pair: the o-projection's operand
    }
}

// q, k and v of one (row, head) at once: thread t < 192 owns element t % 64 of q / k / v
// (t / 64) and reproduces reduce_head's summation order exactly (per-wave slab sums
// s = w, w+4, ... then bias + (((w0 + w1) + w2) + w3)), so the result is bit-identical
// to three reduce_head calls, in one round trip and one barrier instead of three and six.
// q/k/v element t (< 3 * HD) of head h: bias + the split-K slabs summed as four chains
// (chain w: slabs w, w+4 pairwise by 8, then the chains in order).  QkvLoad issues every
// load up front (ks <= 16: one round trip; clamped addresses, the surplus unused) so the
// kernel can test the row's state meanwhile; qkv_finish sums in the same order for any ks.
struct QkvLoad {
    float p[16];
    float bias;
};
template <bool DEV = false>
__device__ __forceinline__ void qkv_load(const float* __restrict__ part, int ks, int64_t slab, int64_t row, int D,
                                         int h, const float* __restrict__ bias, QkvLoad& L) {
    const int t = threadIdx.x;
    if (t < 3 * HD) {
        const int which = t >> 6, d = t & 63;
        const int64_t off = row + which * D + h * HD + d;
        L.bias = bias[which * D + h * HD + d];
        if (ks <= 16) {
#pragma unroll
            for (int j = 0; j < 16; ++j) L.p[j] = ldslab<DEV>(part + min(j, ks - 1) * slab + off);
        }
    }
}
template <bool DEV = false>
__device__ __forceinline__ void qkv_finish(const float* __restrict__ part, int ks, int64_t slab, int64_t row, int D,
                                           int h, const QkvLoad& L, h16* q16, h16* kdst, h16* vdst) {
    const int t = threadIdx.x;
    if (t < 3 * HD) {
        const int which = t >> 6, d = t & 63;
        const int64_t off = row + which * D + h * HD + d;
        float ws[4];
        if (ks <= 16) {
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                float v = 0.f;
                if (w + 4 < ks) v += L.p[w] + L.p[w + 4];
                else if (w < ks) v += L.p[w];
                if (w + 12 < ks) v += L.p[w + 8] + L.p[w + 12];
                else if (w + 8 < ks) v += L.p[w + 8];
                ws[w] = v;
            }
        } else {
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                float v = 0.f;
                int s = w;
                for (; s + 4 < ks; s += 8) v += ldslab<DEV>(part + s * slab + off) + ldslab<DEV>(part + (s + 4) * slab + off);
                if (s < ks) v += ldslab<DEV>(part + s * slab + off);
                ws[w] = v;
            }
        }
        float r = L.bias;
        r += ws[0] + ws[1] + ws[2] + ws[3];
        h16* dst = which == 0 ? q16 : which == 1 ? kdst : vdst;
        dst[d] = (h16)r;
    }
}

// One (row b, head h) of the plain (non-beam) self-attention: q, k, v from the qkv
// projection's split-K slabs + bias, k and v appended to the cache at the row's position,
// then attend over positions 0..pos.  A finished row reads and writes nothing more.
// DEV: the slabs come from other workgroups of the calling launch (TAIL_ATTN).
template <bool VPRE, bool DEV, bool KALL = false>
__device__ __forceinline__ void self_attn_one(const float* __restrict__ part, int ks, const float* __restrict__ bias,
                                              h16* __restrict__ kcache, h16* __restrict__ vcache,
                                              const int* __restrict__ pos_ptr, int H, int B, int ctx,
                                              h16* __restrict__ out, int64_t lo_off, const SelState* __restrict__ st,
                                              int pos_row, int b, int h) {
    __shared__ h16 q16[HD];
    const int done = st[b].done;
    const int D = H * HD;
    // graph replays may run past max_length on finished windows; pos_row: per-row counters (row refill)
    const int pos = min(pos_ptr[pos_row ? b : 0], ctx - 1);
    const int64_t slab = (int64_t)B * 3 * D, row = (int64_t)b * 3 * D;
    QkvLoad L;
    qkv_load<DEV>(part, ks, slab, row, D, h, bias, L);
    if (done) return;
    h16* kc = kcache + ((int64_t)b * H + h) * ctx * HD;
    h16* vc = vcache + ((int64_t)b * H + h) * ctx * HD;
    qkv_finish<DEV>(part, ks, slab, row, D, h, L, q16, kc + (int64_t)pos * HD, vc + (int64_t)pos * HD);
    __threadfence_block();
    __syncthreads();
    attend_one<448, false, true, VPRE, KALL>(q16, kc, vc, pos + 1, out + (int64_t)b * D + h * HD, lo_off);
}
