// Shared device/host helpers for the gfx950 kernels of libosw_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

namespace osw {

typedef _Float16 h16;
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 h16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((vector_size(8)));

#define OSW_LDS __attribute__((address_space(3)))

// ordered-int encoding so atomicMax on int orders floats (incl. negatives)
__device__ __forceinline__ int float_to_ordered(float f) {
    int i = __float_as_int(f);
    return i >= 0 ? i : (i ^ 0x7fffffff);
}
__device__ __forceinline__ float ordered_to_float(int i) {
    return __int_as_float(i >= 0 ? i : (i ^ 0x7fffffff));
}

// erf(x) to |error| <= 1.5e-7 (Abramowitz & Stegun 7.1.26): one reciprocal, one exp,
// five FMAs and no branches.  ocml's erff takes a divergent two-branch path that made
// the GELU epilogue of the encoder fc1 GEMM ~30 % of that kernel's time; the result
// is stored as fp16 (relative step 4.9e-4), far above this error.
__device__ __forceinline__ float erf_fast(float x) {
    const float ax = fabsf(x);
    const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
    float y = fmaf(fmaf(fmaf(fmaf(1.061405429f, t, -1.453152027f), t, 1.421413741f), t, -0.284496736f), t,
                   0.254829592f) * t;
    y = 1.0f - y * __expf(-ax * ax);
    return copysignf(y, x);
}

// The result is rounded to fp32 before any fp16 conversion: without the opaque move the
// compiler fused the last multiply into the conversion (v_fma_mixlo_f16, one rounding) in
// some epilogues and not in others (v_mul_f32 + v_cvt_pk_f16_f32), so the same GELU
// input could leave two tile kernels as different fp16 values
__device__ __forceinline__ float gelu_erf(float x) {
    float r = 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f));
    asm("" : "+v"(r));
    return r;
}

// Lane exchange v[lane ^ O] without the LDS pipe: DPP for O <= 8 (quad_perm, half-row
// mirror + quad reverse for 4, row rotate for 8), gfx950's v_permlane{16,32}_swap for
// 16 / 32.  ds_bpermute (what __shfl_xor lowers to) with several permutes in flight
// returned stale lanes when another queue's LDS-DMA kernels shared the CU (the decoder
// of one context drifted while a second context encoded; DESIGN.md "Determinism"),
// and DPP is also a few cycles instead of an LDS round trip.
template <int V>
using IC = std::integral_constant<int, V>;
template <int O>
__device__ __forceinline__ int xor_lane(int v) {
    static_assert(O == 1 || O == 2 || O == 4 || O == 8 || O == 16 || O == 32, "xor distance");
    if constexpr (O == 1) {
        return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
    } else if constexpr (O == 2) {
        return __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
    } else if constexpr (O == 4) {
        const int t = __builtin_amdgcn_update_dpp(0, v, 0x141, 0xf, 0xf, false);  // row_half_mirror: i -> 7-i
        return __builtin_amdgcn_update_dpp(0, t, 0x1B, 0xf, 0xf, false);          // quad_perm [3,2,1,0]
    } else if constexpr (O == 8) {
        return __builtin_amdgcn_update_dpp(0, v, 0x128, 0xf, 0xf, false);  // row_ror:8 == xor 8 in a 16-lane row
    } else if constexpr (O == 16) {
        // (v, v) -> first = rows [0,0,2,2], second = rows [1,1,3,3]
        const auto r = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
        return (int)((__lane_id() & 16) ? r[0] : r[1]);
    } else {
        // (v, v) -> first = halves [lo,lo], second = [hi,hi]
        const auto r = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
        return (int)((__lane_id() & 32) ? r[0] : r[1]);
    }
}
template <int O>
__device__ __forceinline__ float xor_lane(float v) {
    return __int_as_float(xor_lane<O>(__float_as_int(v)));
}

__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, xor_lane<32>(v));
    v = fmaxf(v, xor_lane<16>(v));
    v = fmaxf(v, xor_lane<8>(v));
    v = fmaxf(v, xor_lane<4>(v));
    v = fmaxf(v, xor_lane<2>(v));
    return fmaxf(v, xor_lane<1>(v));
}
__device__ __forceinline__ float wave_sum(float v) {
    v += xor_lane<32>(v);
    v += xor_lane<16>(v);
    v += xor_lane<8>(v);
    v += xor_lane<4>(v);
    v += xor_lane<2>(v);
    return v + xor_lane<1>(v);
}

// GEMM epilogue selector (see gemm.hip)
enum Epi : int {
    EPI_F16 = 0,          // C16 = acc + bias
    EPI_F16_GELU = 1,     // C16 = gelu(acc + bias)
    EPI_F32_RESID = 2,    // C32 += acc + bias          (residual stream, in place)
    EPI_F32_GELU_POS = 3, // C32 = gelu(acc + bias) + pos[t]   (conv2 -> residual)
    EPI_F32 = 4,          // C32 = acc + bias           (logits)
    EPI_HEADS = 5,        // C16 head-major [which][nb][H][T][64] = acc + bias
};

struct GemmArgs {
    const h16* A; int64_t lda; int64_t a_grp_rows; int64_t a_grp_stride;
    const h16* W; int64_t ldw;           // W[N][K]
    const float* bias;                   // [N] or nullptr
    int M, N, K;
    void* C; int64_t ldc; int64_t c_grp_rows; int64_t c_grp_stride;
    const float* pos;                    // EPI_F32_GELU_POS: pos[(m % c_grp_rows)][n]
    int epi;
    int heads_T, heads_H, heads_nb;      // EPI_HEADS geometry
    const int* heads_slot;               // EPI_HEADS: window b of this GEMM goes to slot heads_slot[b] (nullptr: b)
    int band;                            // 256-tile walk: column band width (0 = all columns)
    int kc;                              // 128-tile split-K: K per blockIdx.z, EPI_F32 slab z at C + z*M*ldc (0 = K)
    // decoder activations as an fp16 pair a = hi + lo (hi = fp16(a), lo = fp16(a - hi)):
    // A_lo has A's row addressing; the kernels accumulate hi·W then lo·W into the same
    // fp32 accumulators, so the product carries ~22 bits of the fp32 activation.
    // nullptr: A alone (fp16 activations).  Supported by the skinny and wide kernels (the
    // decoder's); launch_gemm routes every A_lo GEMM to them.
    const h16* A_lo;
    // skinny kernel, hi/lo rows in 32-row groups: issue every k32 step of the workgroup's
    // weights up front (kc <= 256) instead of one chunk ahead (set by the launcher)
    int preload_w;
    // skinny kernel, several row groups: a 1-D grid where the row groups of one (column
    // block, K range) are consecutive workgroups of one XCD (ids 8j + x, j = row group
    // fastest), so the second group's weight reads hit the L2 the first one filled
    int pair_rows;
    // 8-phase persistent GEMM: 1 = leave a quarter of the CUs to other lanes' kernels (set
    // while sibling contexts have calls in flight), 0 = one workgroup on every CU
    int share_cus;
    // skinny kernel: W's fragment-major copy, [ceil(N/16)][K/32][64 lanes][8] (the 16 x 32
    // MFMA B fragment of one k32 step is 1 KB contiguous, so a wave's weight load is one
    // coalesced 1-KB piece instead of 16 rows x 64 B; launch_frag_pack), or nullptr
    const h16* Wf;
};

// fp32 -> (hi, lo) fp16 pair: hi = fp16(v), lo = fp16(v - hi)
__device__ __forceinline__ void split_h16(float v, h16* hi, h16* lo, int64_t i) {
    const h16 h = (h16)v;
    hi[i] = h;
    lo[i] = (h16)(v - (float)h);
}

// launchers (defined in the .hip files)
void launch_gemm(const GemmArgs& g, hipStream_t s);
// W[N][ldw] (K columns used) -> its fragment-major copy Wf (GemmArgs::Wf), zero past N
void launch_frag_pack(const h16* W, int64_t ldw, int N, int K, h16* Wf, hipStream_t s);
void launch_gemm_variant(const GemmArgs& g, int variant, hipStream_t s);  // 0 auto, 1 128-tile, 2 256-tile,
                                                                          // 4 8-phase 256, 5 wide, 6 64-tile ring, 7 64-tile;
                                                                          // debug: 8 8-phase fp16 out, 9 no epilogue, 10 GELU
// M <= 64, K % 128 == 0; `part` needs skinny_ksplit(N,K)*M*N floats
void launch_gemm_skinny(const GemmArgs& g, float* part, hipStream_t s);
int skinny_ksplit(int N, int K);
void prepare_gemm_kernels();  // every GEMM kernel's dynamic-LDS attribute, once (osw_create)
int tiled_ksplit(int M, int N, int K);
void launch_gemm_tiled_partial(const GemmArgs& g, float* part, int ks, hipStream_t s);
int launch_gemm_skinny_partial(const GemmArgs& g, float* part, hipStream_t s);
struct ProArgs;
int launch_gemm_skinny_gelu_tail(const GemmArgs& g, float* part, const ProArgs& pa, hipStream_t s);
int launch_gemm_skinny_pro(const GemmArgs& g, int pro, const ProArgs& pa, bool direct, float* part, hipStream_t s,
                           bool select = false, bool attn_tail = false);
void launch_layernorm(const float* x, int64_t M, int D, const float* g, const float* b, h16* y, hipStream_t s);

}  // namespace osw
