// Decoder-step kernels (one token per window per step): self-attention over the
// KV cache, cross-attention over the 1500 precomputed encoder K/V, and the greedy
// token selection with Whisper's logits rules.
//
// Cross-attention is the bandwidth hot spot of decoding: each step reads the whole
// K and V of every (window, head): 2 x 1500 x 64 fp16 = 384 KB per (b, h).  One
// workgroup per (b, h); K rows are read 128 B per lane (8 x 16 B), V in 1 KiB
// contiguous wave-instructions (8 rows x 128 B), scores stay in LDS.
#include "common.h"

namespace osw {

namespace {
constexpr int HD = 64;

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

// Attention of one query row over n_keys rows of K/V ([n][64] fp16, contiguous).
// 256 threads.  Scores live in LDS (n_keys <= MAXK).  Loads are issued in groups
// (2 K rows = 16 x 16 B per lane, 8 V pieces per lane) before the FMAs that use
// them so each lane keeps several HBM requests in flight.
template <int MAXK>
__device__ void attend_one(const h16* __restrict__ q16, const h16* __restrict__ K, const h16* __restrict__ V,
                           int n_keys, h16* __restrict__ out) {
    __shared__ float qs[HD];
    __shared__ float sc[MAXK];
    __shared__ float red[8];
    __shared__ f32x4 part[32][17];  // [key group][8 d-chunks x 2 float4]
    const int tid = threadIdx.x;
    if (tid < HD) qs[tid] = (float)q16[tid] * 0.125f;  // 1/sqrt(64), exact in fp32
    __syncthreads();
    float q[HD];
#pragma unroll
    for (int i = 0; i < HD; ++i) q[i] = qs[i];
    float mx = -INFINITY;
    for (int j0 = tid; j0 < n_keys; j0 += 512) {
        const int j1 = j0 + 256;
        const bool two = j1 < n_keys;
        const h16x8* k0 = (const h16x8*)(K + (int64_t)j0 * HD);
        const h16x8* k1 = (const h16x8*)(K + (int64_t)(two ? j1 : j0) * HD);
        h16x8 a[8], b[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) a[c] = k0[c];
#pragma unroll
        for (int c = 0; c < 8; ++c) b[c] = k1[c];
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                s0 = fmaf((float)a[c][j], q[8 * c + j], s0);
                s1 = fmaf((float)b[c][j], q[8 * c + j], s1);
            }
        sc[j0] = s0;
        mx = fmaxf(mx, s0);
        if (two) {
            sc[j1] = s1;
            mx = fmaxf(mx, s1);
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
    // PV: thread -> (key group kg = tid>>3, d chunk c = tid&7), keys j = kg + 32 i;
    // one wave-instruction reads 8 consecutive V rows = 1 KiB contiguous
    const int kg = tid >> 3, c = tid & 7;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int j = kg;
    for (; j + 32 * 7 < n_keys; j += 32 * 8) {
        h16x8 v[8];
        float p[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = *(const h16x8*)(V + (int64_t)(j + 32 * u) * HD + 8 * c);
#pragma unroll
        for (int u = 0; u < 8; ++u) p[u] = sc[j + 32 * u];
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[e] = fmaf(p[u], (float)v[u][e], acc[e]);
    }
    for (; j < n_keys; j += 32) {
        const h16x8 v = *(const h16x8*)(V + (int64_t)j * HD + 8 * c);
        const float p = sc[j];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = fmaf(p, (float)v[e], acc[e]);
    }
    part[kg][2 * c] = f32x4{acc[0], acc[1], acc[2], acc[3]};
    part[kg][2 * c + 1] = f32x4{acc[4], acc[5], acc[6], acc[7]};
    __syncthreads();
    if (tid < HD) {
        const int cc = tid >> 3, e = tid & 7;
        float r = 0.f;
        for (int k = 0; k < 32; ++k) r += part[k][2 * cc + (e >> 2)][e & 3];
        out[tid] = (h16)(r / sum);
    }
}

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
// appended to the cache at the device-side position; attend over 0..pos.
__global__ __launch_bounds__(256) void dec_self_attn_kernel(const float* __restrict__ part, int ks,
                                                            const float* __restrict__ bias, h16* __restrict__ kcache,
                                                            h16* __restrict__ vcache, const int* __restrict__ pos_ptr,
                                                            int H, int B, int ctx, h16* __restrict__ out) {
    __shared__ h16 q16[HD];
    __shared__ float red4[256];
    const int h = blockIdx.x, b = blockIdx.y;
    const int D = H * HD;
    const int pos = min(*pos_ptr, ctx - 1);  // graph replays may run past max_length on finished windows
    h16* kc = kcache + ((int64_t)b * H + h) * ctx * HD;
    h16* vc = vcache + ((int64_t)b * H + h) * ctx * HD;
    const int64_t slab = (int64_t)B * 3 * D, row = (int64_t)b * 3 * D;
    reduce_head(part, ks, slab, row + h * HD, bias, h * HD, q16, red4);
    reduce_head(part, ks, slab, row + D + h * HD, bias, D + h * HD, kc + (int64_t)pos * HD, red4);
    reduce_head(part, ks, slab, row + 2 * D + h * HD, bias, 2 * D + h * HD, vc + (int64_t)pos * HD, red4);
    __threadfence_block();
    __syncthreads();
    attend_one<448>(q16, kc, vc, pos + 1, out + (int64_t)b * D + h * HD);
}

// grid (H, B): q = Σ split-K partials of the cross-attention q projection + bias;
// xkv layer slice: K at ((b*H + h)*T*64) of xk, V likewise of xv
__global__ __launch_bounds__(256) void dec_cross_attn_kernel(const float* __restrict__ part, int ks,
                                                             const float* __restrict__ bias,
                                                             const h16* __restrict__ xk, const h16* __restrict__ xv,
                                                             int H, int B, int T, h16* __restrict__ out) {
    __shared__ h16 q16[HD];
    __shared__ float red4[256];
    const int h = blockIdx.x, b = blockIdx.y;
    const int D = H * HD;
    reduce_head(part, ks, (int64_t)B * D, (int64_t)b * D + h * HD, bias, h * HD, q16, red4);
    const int64_t hoff = ((int64_t)b * H + h) * T * HD;
    attend_one<1536>(q16, xk + hoff, xv + hoff, T, out + (int64_t)b * D + h * HD);
}

// grid B, 1024 threads: x[b] += bias + Σ split-K partials (residual stream, fp32),
// then LayerNorm(x[b]) -> y[b] fp16 (the next projection's operand).  Each thread
// owns <= 2 columns and keeps 4 slab loads in flight.  With part == nullptr it is
// the embedding entry: x[b] = tok_emb[tok[b]] + pos_emb[pos].
__global__ __launch_bounds__(1024) void dec_resid_ln_kernel(const float* __restrict__ part, int ks, int B, int D,
                                                            const float* __restrict__ bias, float* __restrict__ x,
                                                            const float* __restrict__ g, const float* __restrict__ be,
                                                            h16* __restrict__ y, const h16* __restrict__ tok_emb,
                                                            const float* __restrict__ pos_emb,
                                                            const int* __restrict__ tok,
                                                            const int* __restrict__ pos_ptr, int ctx) {
    __shared__ float red[16];
    const int b = blockIdx.x, tid = threadIdx.x;
    constexpr int PER = 2;  // D <= 2048
    float v[PER];
    float s = 0.f;
    const int64_t slab = (int64_t)B * D, rb = (int64_t)b * D;
    int t = 0, pos = 0;
    if (!part) {
        t = tok[b];
        pos = min(*pos_ptr, ctx - 1);
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int c = tid + 1024 * i;
        float a = 0.f;
        if (c < D) {
            if (part) {
                float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
                int k = 0;
                for (; k + 3 < ks; k += 4) {
                    a0 += part[(k + 0) * slab + rb + c];
                    a1 += part[(k + 1) * slab + rb + c];
                    a2 += part[(k + 2) * slab + rb + c];
                    a3 += part[(k + 3) * slab + rb + c];
                }
                for (; k < ks; ++k) a0 += part[k * slab + rb + c];
                a = x[rb + c] + (bias ? bias[c] : 0.f) + ((a0 + a1) + (a2 + a3));
            } else {
                a = (float)tok_emb[(int64_t)t * D + c] + pos_emb[(int64_t)pos * D + c];
            }
            x[rb + c] = a;
        }
        v[i] = a;
        s += a;
    }
    const float mean = block_reduce_sum(s, red) / D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int c = tid + 1024 * i;
        if (c < D) q += (v[i] - mean) * (v[i] - mean);
    }
    const float rstd = rsqrtf(block_reduce_sum(q, red) / D + 1e-5f);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int c = tid + 1024 * i;
        if (c < D) y[rb + c] = (h16)((v[i] - mean) * rstd * g[c] + be[c]);
    }
}

// fc1: h[b][n] = fp16(gelu(bias + Σ partials))
__global__ __launch_bounds__(256) void dec_reduce_gelu_kernel(const float* __restrict__ part, int ks, int64_t total,
                                                              int N, const float* __restrict__ bias,
                                                              h16* __restrict__ y) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        float v = bias[i % N];
        for (int k = 0; k < ks; ++k) v += part[k * total + i];
        y[i] = (h16)gelu_erf(v);
    }
}

// ---------------------------------------------------------------------------
// Greedy selection.  Per-window state lives in device memory so a step needs no
// host round trip.
struct SelState {
    int n_sampled, last, penult, last_ts, done, lang;
    float sum_lp, nsp;
};

struct SelParams {
    int prompt_len;        // P: positions 0..P-1 are prompt
    int sot_pos;           // position of <|startoftranscript|> in the prompt
    int lang_pos;          // prompt position holding the language token (-1 placeholder => detect)
    int max_length;
    int V, eot, no_speech, no_ts, tb, blank, first_lang, n_langs;
    int suppress_blank, with_ts, max_init_ts;
};

struct ArgMax {
    float v;
    int i;
};
__device__ __forceinline__ ArgMax amax(ArgMax a, ArgMax b) {
    return (b.v > a.v || (b.v == a.v && b.i < a.i)) ? b : a;
}
__device__ __forceinline__ void lse_add(float& m, float& s, float x) {  // online log-sum-exp
    if (x == -INFINITY) return;
    if (x > m) {
        s = s * __expf(m - x) + 1.f;
        m = x;
    } else {
        s += __expf(x - m);
    }
}
__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
    if (m2 == -INFINITY) return;
    if (m == -INFINITY) { m = m2; s = s2; return; }
    if (m2 > m) { s = s * __expf(m - m2) + s2; m = m2; }
    else s += s2 * __expf(m2 - m);
}

__global__ __launch_bounds__(1024) void select_kernel(const float* __restrict__ logits, SelParams P,
                                                      const int* __restrict__ pos_ptr,  // position just computed
                                                      const int* __restrict__ prompt,   // [B][P] (-1 = detect)
                                                      const unsigned* __restrict__ supmask,  // V bits
                                                      SelState* __restrict__ st, int* __restrict__ cur_tok,
                                                      int* __restrict__ tokens, int max_tokens) {
    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const float* x = logits + (int64_t)b * P.V;
    __shared__ float rm[16], rs[16], rm2[16], rs2[16];
    __shared__ ArgMax ra[16], ra2[16], ra3[16];
    SelState s = st[b];
    const int w = tid >> 6, l = tid & 63;
    const int step = *pos_ptr;

    if (step < P.prompt_len - 1) {
        // prompt step: forced next token; SOT position -> no-speech prob (+ language detection)
        int next = prompt[b * P.prompt_len + step + 1];
        if (step == P.sot_pos) {
            float m = -INFINITY, sum = 0.f;
            ArgMax best{-INFINITY, 0x7fffffff};
            for (int v = tid; v < P.V; v += blockDim.x) {
                const float xv = x[v];
                lse_add(m, sum, xv);
                if (v >= P.first_lang && v < P.first_lang + P.n_langs) best = amax(best, ArgMax{xv, v});
            }
            // reduce
            for (int o = 32; o > 0; o >>= 1) {
                const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(sum, o, 64);
                lse_merge(m, sum, m2, s2);
                ArgMax bb{__shfl_xor(best.v, o, 64), __shfl_xor(best.i, o, 64)};
                best = amax(best, bb);
            }
            if (l == 0) { rm[w] = m; rs[w] = sum; ra[w] = best; }
            __syncthreads();
            if (tid == 0) {
                float M = rm[0], S = rs[0];
                ArgMax B = ra[0];
                for (int i = 1; i < (int)(blockDim.x >> 6); ++i) { lse_merge(M, S, rm[i], rs[i]); B = amax(B, ra[i]); }
                const float lse = M + __logf(S);
                s.nsp = __expf(x[P.no_speech] - lse);
                if (next < 0) next = B.i;
                s.lang = next;
                st[b] = s;
                cur_tok[b] = next;
            }
            return;
        }
        if (tid == 0) cur_tok[b] = next < 0 ? s.lang : next;
        return;
    }

    if (s.done) {
        if (tid == 0) cur_tok[b] = P.eot;
        return;
    }
    // ---- sampling step: masks are applied on the fly
    const int n = s.n_sampled;
    const bool last_ts = n >= 1 && s.last >= P.tb;
    const bool pen_ts = n < 2 || s.penult >= P.tb;
    int ts_lo_block = P.tb;  // timestamps in [tb, ts_min) are forbidden
    if (P.with_ts && s.last_ts > 0) ts_lo_block = (last_ts && !pen_ts) ? s.last_ts : s.last_ts + 1;
    float m_all = -INFINITY, s_all = 0.f, m_ts = -INFINITY, s_ts = 0.f;
    ArgMax a_all{-INFINITY, 0x7fffffff}, a_text{-INFINITY, 0x7fffffff}, a_ts{-INFINITY, 0x7fffffff};
    for (int v = tid; v < P.V; v += blockDim.x) {
        float xv = x[v];
        bool masked = (supmask[v >> 5] >> (v & 31)) & 1u;
        if (P.suppress_blank && n == 0 && (v == P.blank || v == P.eot)) masked = true;
        if (P.with_ts) {
            if (v == P.no_ts) masked = true;
            if (last_ts) {
                if (pen_ts) { if (v >= P.tb) masked = true; }
                else { if (v < P.eot) masked = true; }
            }
            if (v >= P.tb && v < ts_lo_block) masked = true;
            if (n == 0) {
                if (v < P.tb) masked = true;
                if (P.max_init_ts >= 0 && v > P.tb + P.max_init_ts) masked = true;
            }
        }
        if (masked) continue;
        lse_add(m_all, s_all, xv);
        a_all = amax(a_all, ArgMax{xv, v});
        if (v >= P.tb) {
            lse_add(m_ts, s_ts, xv);
            a_ts = amax(a_ts, ArgMax{xv, v});
        } else {
            a_text = amax(a_text, ArgMax{xv, v});
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        float m2 = __shfl_xor(m_all, o, 64), s2 = __shfl_xor(s_all, o, 64);
        lse_merge(m_all, s_all, m2, s2);
        m2 = __shfl_xor(m_ts, o, 64); s2 = __shfl_xor(s_ts, o, 64);
        lse_merge(m_ts, s_ts, m2, s2);
        a_all = amax(a_all, ArgMax{__shfl_xor(a_all.v, o, 64), __shfl_xor(a_all.i, o, 64)});
        a_text = amax(a_text, ArgMax{__shfl_xor(a_text.v, o, 64), __shfl_xor(a_text.i, o, 64)});
        a_ts = amax(a_ts, ArgMax{__shfl_xor(a_ts.v, o, 64), __shfl_xor(a_ts.i, o, 64)});
    }
    if (l == 0) { rm[w] = m_all; rs[w] = s_all; rm2[w] = m_ts; rs2[w] = s_ts; ra[w] = a_all; ra2[w] = a_text; ra3[w] = a_ts; }
    __syncthreads();
    if (tid == 0) {
        float MA = rm[0], SA = rs[0], MT = rm2[0], ST = rs2[0];
        ArgMax A = ra[0], AX = ra2[0], AT = ra3[0];
        for (int i = 1; i < (int)(blockDim.x >> 6); ++i) {
            lse_merge(MA, SA, rm[i], rs[i]);
            lse_merge(MT, ST, rm2[i], rs2[i]);
            A = amax(A, ra[i]); AX = amax(AX, ra2[i]); AT = amax(AT, ra3[i]);
        }
        const float lse_all = MA + __logf(SA);
        int next = A.i;
        float lp = A.v - lse_all;
        if (P.with_ts) {
            const float lse_ts = MT == -INFINITY ? -INFINITY : MT + __logf(ST);
            const float ts_lp = lse_ts - lse_all;
            const float text_lp = AX.v - lse_all;
            if (ts_lp > text_lp) {  // timestamp mass wins: text suppressed, renormalise over timestamps
                next = AT.i;
                lp = AT.v - lse_ts;
            }
        }
        s.sum_lp += lp;
        if (next == P.eot) {
            s.done = 1;
        } else {
            if (n < max_tokens) tokens[(int64_t)b * max_tokens + n] = next;
            s.n_sampled = n + 1;
            s.penult = s.last;
            s.last = next;
            if (next >= P.tb) s.last_ts = next;
            if (P.prompt_len + s.n_sampled >= P.max_length) s.done = 1;
        }
        st[b] = s;
        cur_tok[b] = next;
    }
}

__global__ void count_done_kernel(const SelState* st, int B, int* out) {
    int c = 0;
    for (int i = threadIdx.x; i < B; i += blockDim.x) c += st[i].done;
    c = (int)wave_sum((float)c);
    if (threadIdx.x == 0) *out = c;
}

__global__ void bump_kernel(int* p) { *p += 1; }
}  // namespace

int sel_state_bytes() { return (int)sizeof(SelState); }

void launch_dec_self_attn(const float* part, int ks, const float* bias, h16* kc, h16* vc, const int* pos, int B,
                          int H, int ctx, h16* out, hipStream_t s) {
    dec_self_attn_kernel<<<dim3(H, B), 256, 0, s>>>(part, ks, bias, kc, vc, pos, H, B, ctx, out);
}

void launch_dec_cross_attn(const float* part, int ks, const float* bias, const h16* xk, const h16* xv, int B, int H,
                           int T, h16* out, hipStream_t s) {
    dec_cross_attn_kernel<<<dim3(H, B), 256, 0, s>>>(part, ks, bias, xk, xv, H, B, T, out);
}

void launch_dec_resid_ln(const float* part, int ks, int B, int D, const float* bias, float* x, const float* g,
                         const float* be, h16* y, const h16* tok_emb, const float* pos_emb, const int* tok,
                         const int* pos, int ctx, hipStream_t s) {
    dec_resid_ln_kernel<<<B, 1024, 0, s>>>(part, ks, B, D, bias, x, g, be, y, tok_emb, pos_emb, tok, pos, ctx);
}

void launch_dec_reduce_gelu(const float* part, int ks, int B, int N, const float* bias, h16* y, hipStream_t s) {
    const int64_t total = (int64_t)B * N;
    dec_reduce_gelu_kernel<<<(unsigned)std::min<int64_t>((total + 255) / 256, 1024), 256, 0, s>>>(part, ks, total, N,
                                                                                                 bias, y);
}

void launch_select(const float* logits, int B, const int* pos, int prompt_len, int sot_pos, int lang_pos,
                   int max_length, int V, int eot, int no_speech, int no_ts, int tb, int blank, int first_lang,
                   int n_langs, int suppress_blank, int with_ts, int max_init_ts, const int* prompt,
                   const unsigned* supmask, void* st, int* cur_tok, int* tokens, int max_tokens, hipStream_t s) {
    SelParams P{prompt_len, sot_pos, lang_pos, max_length, V, eot, no_speech, no_ts, tb, blank, first_lang,
                n_langs, suppress_blank, with_ts, max_init_ts};
    select_kernel<<<B, 1024, 0, s>>>(logits, P, pos, prompt, supmask, (SelState*)st, cur_tok, tokens, max_tokens);
}

void launch_count_done(const void* st, int B, int* out, hipStream_t s) {
    count_done_kernel<<<1, 64, 0, s>>>((const SelState*)st, B, out);
}

void launch_bump(int* p, hipStream_t s) { bump_kernel<<<1, 1, 0, s>>>(p); }

}  // namespace osw
