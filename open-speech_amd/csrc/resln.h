// Decoder residual update + LayerNorm, in the ONE formulation that both the standalone
// kernel (decode.hip, dec_resid_ln_kernel) and the fused prologue of the small-batch
// decoder GEMM (gemm.hip, gemm_skinny_kernel<.., PRO>) run, so a window's results do not
// depend on which of the two paths its batch size selected (bit-identical by
// construction; tests/test_gpu_parity.py::test_batch_equals_single).
//
// Per row r:  x' = x + bias + Σ_k part[k][r]   (or the embedding tok_emb[tok] + pos_emb[pos])
//             y  = (x' - mean) * rstd * g + b   (two-pass variance, eps 1e-5, fp32)
// 256 threads; thread t owns columns 4t..4t+3 (one 16-B piece) and 1024 + t (D <= 1280).
// Every slab piece of a row is loaded before any is added (8 slabs per batch, clamped
// addresses, the surplus added as exact zeros), with the residual, bias, gain and shift
// issued ahead of the first batch, so a row costs one memory round trip per 8 slabs; the sums run in slab order, the thread's 5 columns in order, then
// wave_sum, then the 4 wave partials in order.
#pragma once
#include "common.h"
#include "decode.h"

namespace osw {

struct ResLnArgs {
    const float* part;  // split-K slabs [ks][rows][D]; nullptr = embedding entry
    int ks;
    int64_t slab;       // floats per slab
    const float* bias;  // may be nullptr
    const float* x_in;  // residual stream [rows][D]
    float* x_out;       // updated residual stream (may alias x_in in the standalone kernel)
    const float* g;
    const float* b;
    const h16* tok_emb;  // embedding entry: x' = tok_emb[tok[r]] + pos_emb[min(pos, ctx-1)]
    const float* pos_emb;
    const int* tok;
    const int* pos;
    int ctx;
    int D;
    int V;              // rows of tok_emb: an id outside [0, V) is clamped into it
    int pos_row;        // 1: row r's position is pos[r] (row refill), 0: every row's is pos[0]
};

// rows r0 .. r0+nr-1 (nr <= NR); emit(r, c, y) receives every LayerNorm output;
// write_x: this workgroup stores x'.  red: LDS scratch of 2 * NR * 4 floats.  KB: slab
// loads per batch (the sums do not depend on it: the padding adds exact zeros).  EARLY:
// the residual, bias, gain and shift are loaded ahead of the first slab batch (one round
// trip fewer, ~15 more VGPRs); otherwise after the slabs / the statistics.  Same arithmetic.
template <int NR, int KB, bool EARLY, class Emit>
__device__ __forceinline__ void resln_rows(const ResLnArgs& A, int r0, int nr, bool write_x, float* red, Emit emit) {
#pragma clang fp contract(off)
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const int D = A.D;
    const bool h4 = 4 * t < D, h1 = 1024 + t < D;
    const int c4 = h4 ? 4 * t : 0, c1 = h1 ? 1024 + t : 0;  // clamped: every load stays in the row
    // issued before the first slab batch, so they share its round trip: the LayerNorm gain
    // and shift, the bias, every row's residual (all rows' loads precede any x' store, so
    // x_out aliasing x_in is harmless)
    f32x4 g4, b4, bias4 = {0.f, 0.f, 0.f, 0.f}, x4[NR];
    float g1, b1, bias1 = 0.f, x1[NR];
    auto load_gb = [&]() {
        g4 = *(const f32x4*)(A.g + c4);
        b4 = *(const f32x4*)(A.b + c4);
        g1 = A.g[c1];
        b1 = A.b[c1];
    };
    auto load_x = [&]() {
        if (A.bias) {
            bias4 = *(const f32x4*)(A.bias + c4);
            bias1 = A.bias[c1];
        }
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int64_t rb = (int64_t)(r0 + min(r, nr - 1)) * D;
            x4[r] = *(const f32x4*)(A.x_in + rb + c4);
            x1[r] = A.x_in[rb + c1];
        }
    };
    if constexpr (EARLY) {
        load_gb();
        if (A.part) load_x();
    }
    float v[NR][5];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
#pragma unroll
        for (int i = 0; i < 5; ++i) v[r][i] = 0.f;
        if (r >= nr) continue;
        const int64_t rb = (int64_t)(r0 + r) * D;
        f32x4 a4;
        float a1;
        if (A.part) {
            f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
            float s1 = 0.f;
            for (int k0 = 0; k0 < A.ks; k0 += KB) {
                f32x4 p4[KB];
                float p1[KB];
#pragma unroll
                for (int j = 0; j < KB; ++j) {
                    const int64_t o = (int64_t)min(k0 + j, A.ks - 1) * A.slab + rb;
                    p4[j] = *(const f32x4*)(A.part + o + c4);
                    p1[j] = A.part[o + c1];
                }
#pragma unroll
                for (int j = 0; j < KB; ++j) {
                    const bool in = k0 + j < A.ks;
                    s4 += in ? p4[j] : f32x4{0.f, 0.f, 0.f, 0.f};
                    s1 += in ? p1[j] : 0.f;
                }
            }
            if constexpr (!EARLY)
                if (r == 0) load_x();
            a4 = x4[r];
            a1 = x1[r];
            if (A.bias) {
                a4 += bias4;
                a1 += bias1;
            }
            a4 += s4;
            a1 += s1;
        } else {
            const int tk = min(max(A.tok[r0 + r], 0), A.V - 1);  // defence in depth: select never emits one
            const h16x4 e4 = *(const h16x4*)(A.tok_emb + (int64_t)tk * D + c4);
            const int pos = min(A.pos[A.pos_row ? r0 + r : 0], A.ctx - 1);
            const float* pe = A.pos_emb + (int64_t)pos * D;
            a4 = f32x4{(float)e4[0], (float)e4[1], (float)e4[2], (float)e4[3]} + *(const f32x4*)(pe + c4);
            a1 = (float)A.tok_emb[(int64_t)tk * D + c1] + pe[c1];
        }
        if (write_x) {
            if (h4) *(f32x4*)(A.x_out + rb + c4) = a4;
            if (h1) A.x_out[rb + c1] = a1;
        }
        if (h4) {
            v[r][0] = a4[0];
            v[r][1] = a4[1];
            v[r][2] = a4[2];
            v[r][3] = a4[3];
        }
        if (h1) v[r][4] = a1;
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 5; ++i) s += v[r][i];
        s = wave_sum(s);
        if (l == 0) red[r * 4 + w] = s;
    }
    __syncthreads();
    float mean[NR], rstd[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        mean[r] = (((red[r * 4 + 0] + red[r * 4 + 1]) + red[r * 4 + 2]) + red[r * 4 + 3]) / D;
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < 5; ++i)
            if (i < 4 ? h4 : h1) {
                const float d = v[r][i] - mean[r];
                q = fmaf(d, d, q);
            }
        q = wave_sum(q);
        if (l == 0) red[(NR + r) * 4 + w] = q;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const float q = (((red[(NR + r) * 4 + 0] + red[(NR + r) * 4 + 1]) + red[(NR + r) * 4 + 2]) +
                         red[(NR + r) * 4 + 3]);
        rstd[r] = rsqrtf(q / D + 1e-5f);
    }
    if constexpr (!EARLY) load_gb();
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        if (r >= nr) break;
        if (h4)
#pragma unroll
            for (int i = 0; i < 4; ++i) emit(r, c4 + i, fmaf((v[r][i] - mean[r]) * rstd[r], g4[i], b4[i]));
        if (h1) emit(r, c1, fmaf((v[r][4] - mean[r]) * rstd[r], g1, b1));
    }
}

// LDS scratch (floats) resln_rows needs for NR rows of D columns
constexpr int resln_scratch(int NR, int D) { return (void)D, 2 * NR * 4; }

// Operand prologue of the small-batch decoder GEMM (gemm.hip): the workgroup builds its
// activation rows itself instead of loading them, so the kernel that produced them
// (residual+LayerNorm, GELU reduce) is not launched at all.
enum Pro : int { PRO_NONE = 0, PRO_RESLN = 1, PRO_GELU = 2 };
constexpr int PRO_ROWS = 1;      // rows the prologue serves: batch-1 latency (every workgroup
                                 // re-reads all rows' slabs, so 5 beam rows were slower, measured)
constexpr int PRO_STRIDE = 1288; // halfs per LDS image row (D <= 1280; +8 staggers the banks)
constexpr int GELU_ROWS = 8;     // PRO_GELU serves up to 8 rows: each workgroup reduces only its
constexpr int GELU_KC = 256;     // own K range (<= GELU_KC deep), so no slab is read twice
// TAIL_ATTN: the batch-1 self-attention run by the qkv GEMM's last arriver per head
// (dec_self_attn_kernel's arguments; the slabs are the GEMM's own)
struct SelfAttnTail {
    const float* bias;   // qkv bias [3D]
    h16* kc;             // this layer's self-K/V cache
    h16* vc;
    const int* pos;
    int H, ctx, pos_row;
    h16* out;            // attention output (hi; lo at out + lo_off)
    int64_t lo_off;
    const SelState* st;
};
struct ProArgs {
    ResLnArgs ln;        // PRO_RESLN: LayerNorm(x') of every row, all D columns
    const float* part;   // PRO_GELU: the fc1 slabs [ks][M][K], K = this GEMM's K
    int ks;
    const float* bias;
    SelFuse sel;         // the batch-1 logits GEMM with the selection in its epilogue (decode.h)
    // TAIL_GELU (split-K partial mode): the last of the ks workgroups of a (64-column block,
    // row group) to finish reduces the block's slabs: y = gelu(bias + Σ_k part[k]) as a
    // hi/lo pair at tail_y[m * N + n] / tail_y[tail_lo + m * N + n], exactly as
    // dec_reduce_gelu_kernel (gelu_reduce_one's order), so that kernel is not launched.
    int* tail_ticket;    // [column blocks x row groups] (TAIL_ATTN: [heads]), zero between launches
    h16* tail_y;
    int64_t tail_lo;
    SelfAttnTail attn;
};
enum Tail : int { TAIL_NONE = 0, TAIL_GELU = 1, TAIL_ATTN = 2 };

// fc1 -> fc2 operand: fp16 pair of gelu(bias + Σ_k part[k][r][n]), k in order (the order of
// dec_reduce_gelu_kernel, which shares this function)
__device__ __forceinline__ float gelu_reduce_one(const float* part, int ks, int64_t slab, const float* bias,
                                                 int64_t i, int n) {
    float v = bias[n];
    for (int k0 = 0; k0 < ks; k0 += 8) {  // 8 slab loads in flight, then the adds in order
        float p[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) p[j] = part[(int64_t)min(k0 + j, ks - 1) * slab + i];
#pragma unroll
        for (int j = 0; j < 8; ++j) v += k0 + j < ks ? p[j] : 0.f;
    }
    return gelu_erf(v);
}

// gelu_reduce_one for NR rows at once (rows past M repeat row M-1): every row's slab loads
// of a batch of 8 slabs are in flight together, the adds per row in gelu_reduce_one's order
template <int NR>
__device__ __forceinline__ void gelu_reduce_rows(const float* part, int ks, int64_t slab, const float* bias, int M,
                                                 int64_t ld, int64_t col, float (&y)[NR]) {
    const float b = bias[col];
#pragma unroll
    for (int r = 0; r < NR; ++r) y[r] = b;
    for (int k0 = 0; k0 < ks; k0 += 8) {
        float p[NR][8];
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
            for (int j = 0; j < 8; ++j) p[r][j] = part[(int64_t)min(k0 + j, ks - 1) * slab + min(r, M - 1) * ld + col];
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
            for (int j = 0; j < 8; ++j) y[r] += k0 + j < ks ? p[r][j] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) y[r] = gelu_erf(y[r]);
}

}  // namespace osw
