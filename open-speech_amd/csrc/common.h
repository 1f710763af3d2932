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

__device__ __forceinline__ float gelu_erf(float x) {
    return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
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
    int band;                            // 256-tile walk: column band width (0 = all columns)
    int kc;                              // 128-tile split-K: K per blockIdx.z, EPI_F32 slab z at C + z*M*ldc (0 = K)
};

// launchers (defined in the .hip files)
void launch_gemm(const GemmArgs& g, hipStream_t s);
void launch_gemm_variant(const GemmArgs& g, int variant, hipStream_t s);  // 0 auto, 1 128-tile, 2 256-tile
// M <= 64, K % 128 == 0; `part` needs skinny_ksplit(N,K)*M*N floats
void launch_gemm_skinny(const GemmArgs& g, float* part, hipStream_t s);
int skinny_ksplit(int N, int K);
int tiled_ksplit(int M, int N, int K);
void launch_gemm_tiled_partial(const GemmArgs& g, float* part, int ks, hipStream_t s);
int launch_gemm_skinny_partial(const GemmArgs& g, float* part, hipStream_t s);
void launch_layernorm(const float* x, int64_t M, int D, const float* g, const float* b, h16* y, hipStream_t s);

}  // namespace osw
