// Row-wise and elementwise kernels: LayerNorm (fp32 residual -> fp16 GEMM
// operand), decoder token+position embedding, and the device-side counter-hash
// weight init (bit-identical to open-speech_amd/weights.py:hash_uniform).
#include "common.h"

#include <cstdlib>

namespace osw {

namespace {
// One wavefront per row; D % 128 == 0 (every Whisper width is); float2 loads.
template <int PER>  // PER = D / 128 float2 per lane
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, int64_t M, int D,
                                                        const float* __restrict__ g, const float* __restrict__ b,
                                                        h16* __restrict__ y) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= M) return;
    const f32x2* xr = (const f32x2*)(x + row * D);
    f32x2 v[PER];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        v[i] = xr[i * 64 + lane];
        s += v[i].x + v[i].y;
    }
    const float mean = wave_sum(s) / D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const float a = v[i].x - mean, c = v[i].y - mean;
        q += a * a + c * c;
    }
    const float rstd = rsqrtf(wave_sum(q) / D + 1e-5f);
    const f32x2* g2 = (const f32x2*)g;
    const f32x2* b2 = (const f32x2*)b;
    h16x2* yr = (h16x2*)(y + row * D);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int c = i * 64 + lane;
        const f32x2 gg = g2[c], bb = b2[c];
        h16x2 o;
        o.x = (h16)((v[i].x - mean) * rstd * gg.x + bb.x);
        o.y = (h16)((v[i].y - mean) * rstd * gg.y + bb.y);
        yr[c] = o;
    }
}

// D % 256 == 0 (base and up; tiny's 384 takes the float2 kernel above): 16-B loads of the
// residual, gamma and beta, 8-B fp16 stores (the float2 form moved 737 MB per turbo encoder
// LayerNorm at ≈ 5.0 TB/s: ten 512-B wave-loads per row and 256-B wave-stores)
template <int PER>  // PER = D / 256 float4 per lane
__global__ __launch_bounds__(256) void layernorm4_kernel(const float* __restrict__ x, int64_t M, int D,
                                                         const float* __restrict__ g, const float* __restrict__ b,
                                                         h16* __restrict__ y) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= M) return;
    const f32x4* xr = (const f32x4*)(x + row * D);
    f32x4 v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) v[i] = __builtin_nontemporal_load(&xr[i * 64 + lane]);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    const float mean = wave_sum(s) / D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const f32x4 a = v[i] - mean;
        q += (a.x * a.x + a.y * a.y) + (a.z * a.z + a.w * a.w);
    }
    const float rstd = rsqrtf(wave_sum(q) / D + 1e-5f);
    const f32x4* g4 = (const f32x4*)g;
    const f32x4* b4 = (const f32x4*)b;
    h16x4* yr = (h16x4*)(y + row * D);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int c = i * 64 + lane;
        const f32x4 gg = g4[c], bb = b4[c];
        h16x4 o;
        o[0] = (h16)((v[i].x - mean) * rstd * gg.x + bb.x);
        o[1] = (h16)((v[i].y - mean) * rstd * gg.y + bb.y);
        o[2] = (h16)((v[i].z - mean) * rstd * gg.z + bb.z);
        o[3] = (h16)((v[i].w - mean) * rstd * gg.w + bb.w);
        __builtin_nontemporal_store(o, &yr[c]);
    }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

template <typename T>
__global__ void init_uniform_kernel(T* dst, int64_t n, uint64_t key, float scale, float offset, int64_t zlo,
                                    int64_t zhi) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t h = splitmix64(key + (uint64_t)i);
        const float u = (float)(h >> 40) * (1.0f / 16777216.0f);
        // same op order as numpy: ((u*2 - 1) * scale) + offset, each rounded to fp32
        const float v = __fadd_rn(__fmul_rn(__fsub_rn(__fmul_rn(u, 2.0f), 1.0f), scale), offset);
        dst[i] = (i >= zlo && i < zhi) ? (T)0.0f : (T)v;
    }
}

__global__ void f16_to_f32_kernel(const h16* __restrict__ a, float* __restrict__ b, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        b[i] = (float)a[i];
}
}  // namespace

void launch_layernorm(const float* x, int64_t M, int D, const float* g, const float* b, h16* y, hipStream_t s) {
    const dim3 grid((unsigned)((M + 3) / 4));
    static const bool f2 = [] {  // OSW_LN_F2=1: the float2 kernel at every width (A/B)
        const char* e = std::getenv("OSW_LN_F2");
        return e && e[0] == '1';
    }();
    if (D % 256 == 0 && !f2) {
        switch (D / 256) {
            case 2: layernorm4_kernel<2><<<grid, 256, 0, s>>>(x, M, D, g, b, y); return;
            case 3: layernorm4_kernel<3><<<grid, 256, 0, s>>>(x, M, D, g, b, y); return;
            case 4: layernorm4_kernel<4><<<grid, 256, 0, s>>>(x, M, D, g, b, y); return;
            case 5: layernorm4_kernel<5><<<grid, 256, 0, s>>>(x, M, D, g, b, y); return;
            default: break;
        }
    }
    switch (D / 128) {
        case 1: layernorm_kernel<1><<<grid, 256, 0, s>>>(x, M, D, g, b, y); break;
        case 2: layernorm_kernel<2><<<grid, 256, 0, s>>>(x, M, D, g, b, y); break;
        case 3: layernorm_kernel<3><<<grid, 256, 0, s>>>(x, M, D, g, b, y); break;
        case 4: layernorm_kernel<4><<<grid, 256, 0, s>>>(x, M, D, g, b, y); break;
        case 6: layernorm_kernel<6><<<grid, 256, 0, s>>>(x, M, D, g, b, y); break;
        case 8: layernorm_kernel<8><<<grid, 256, 0, s>>>(x, M, D, g, b, y); break;
        case 10: layernorm_kernel<10><<<grid, 256, 0, s>>>(x, M, D, g, b, y); break;
        default: layernorm_kernel<10><<<grid, 256, 0, s>>>(x, M, D, g, b, y); break;  // guarded by host check
    }
}

uint64_t hash_stream_key(uint64_t seed, int64_t stream) {
    uint64_t x = seed * 0x632BE59BD9B4E019ull + (uint64_t)stream * 0x2545F4914F6CDD1Dull;
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

void launch_init_uniform(void* dst, bool is_f16, int64_t n, uint64_t key, float scale, float offset, int64_t zlo,
                         int64_t zhi, hipStream_t s) {
    const int blocks = (int)std::min<int64_t>((n + 255) / 256, 8192);
    if (is_f16)
        init_uniform_kernel<h16><<<blocks, 256, 0, s>>>((h16*)dst, n, key, scale, offset, zlo, zhi);
    else
        init_uniform_kernel<float><<<blocks, 256, 0, s>>>((float*)dst, n, key, scale, offset, zlo, zhi);
}


void launch_f16_to_f32(const h16* a, float* b, int64_t n, hipStream_t s) {
    f16_to_f32_kernel<<<1024, 256, 0, s>>>(a, b, n);
}

}  // namespace osw
