// Batch-1 logits GEMV probe: stream a [51866][1280] fp16 weight matrix (the tied token
// embedding) once per launch with the skinny GEMM's access pattern, and with alternatives,
// to see what the 51 us batch-1 logits kernel (133 MB: 22 us at 6 TB/s) is made of.
//   row-major   : lane reads 16 B of column n = lane & 15 at k = 8 (lane >> 4) + 32 st
//                 (a wave instruction touches 16 rows x 64 B), as gemm_skinny_kernel
//   fragment    : the same MFMA B fragments stored fragment-major (16 columns x 32 k =
//                 1 KB contiguous per wave instruction)
//   copy        : a plain float4 stream over the same bytes (the ceiling)
// Three copies of the matrix rotate so the 256 MB MALL cannot serve a launch (the decoder
// streams 317 MB per step).  OCC limits workgroups per CU through dynamic LDS, as the real
// kernel's 166 VGPRs do (3 per CU).
// build: hipcc --offload-arch=gfx950 -O3 -o tools/gemv_probe tools/gemv_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            printf("%s: %s @%d\n", #x, hipGetErrorString(e), __LINE__);                     \
            return 1;                                                                        \
        }                                                                                    \
    } while (0)

typedef _Float16 h16;
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int N = 51866, NP = 51872, K = 1280, NSTEPS = K / 32, CH = 8;

// LAYOUT 0 row-major, 1 fragment-major; CPW 16-column blocks per wave
template <int LAYOUT, int CPW>
__global__ __launch_bounds__(256) void gemv(const h16* __restrict__ W, float* __restrict__ out) {
    extern __shared__ char occ_lds[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    h16x8 a;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = (h16)(0.001f * ((lane + i) & 7));
    const h16* p[CPW];
    int nb[CPW];
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        nb[c] = (blockIdx.x * 4 + wave) * CPW + c;
        const int blk = min(nb[c], NP / 16 - 1);
        if (LAYOUT == 0) p[c] = W + (int64_t)min(blk * 16 + (lane & 15), N - 1) * K + 8 * (lane >> 4);
        else p[c] = W + (int64_t)blk * NSTEPS * 512 + lane * 8;
    }
    constexpr int SS = LAYOUT == 0 ? 32 : 512;  // h16 per k32 step
    f32x4 acc[CPW];
#pragma unroll
    for (int c = 0; c < CPW; ++c) acc[c] = f32x4{0, 0, 0, 0};
    h16x8 wa[CPW][CH], wb[CPW][CH];
    auto load = [&](h16x8 (&w)[CPW][CH], int ch) {
#pragma unroll
        for (int u = 0; u < CH; ++u)
#pragma unroll
            for (int c = 0; c < CPW; ++c) w[c][u] = *(const h16x8*)(p[c] + SS * (ch * CH + u));
    };
    auto use = [&](const h16x8 (&w)[CPW][CH]) {
#pragma unroll
        for (int u = 0; u < CH; ++u)
#pragma unroll
            for (int c = 0; c < CPW; ++c) {
                acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, w[c][u], acc[c], 0, 0, 0);
                acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, w[c][u], acc[c], 0, 0, 0);
            }
    };
    constexpr int NCH = NSTEPS / CH;  // 5
    load(wa, 0);
#pragma unroll
    for (int ch = 0; ch < NCH; ch += 2) {
        if (ch + 1 < NCH) load(wb, ch + 1);
        use(wa);
        if (ch + 1 >= NCH) break;
        if (ch + 2 < NCH) load(wa, ch + 2);
        use(wb);
    }
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
        const int col = nb[c] * 16 + (lane & 15);
        if ((lane >> 4) == 0 && col < N) out[col] = acc[c][0];
    }
    if (occ_lds[0] == 1 && lane == 99) out[0] = 0;  // keeps the LDS allocation
}

__global__ __launch_bounds__(256) void copy_read(const float4* __restrict__ src, int64_t n4, float* out) {
    float4 s = {0, 0, 0, 0};
    constexpr int U = 8;
    for (int64_t i = (int64_t)blockIdx.x * 256 * U + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256 * U) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = src[min(i + 256 * u, n4 - 1)];
#pragma unroll
        for (int u = 0; u < U; ++u) { s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w; }
    }
    if (s.x == 1234.5f) out[blockIdx.x] = s.y + s.z + s.w;
}

template <typename F>
int time_graph(const char* name, hipStream_t s, F&& launch) {
    hipGraph_t g;
    hipGraphExec_t ge;
    const int n = 30;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < n; ++i) launch(i % 3);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 2; ++w) CK(hipGraphLaunch(ge, s));
    const int reps = 5;
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / (reps * n);
    printf("%-52s %7.2f us per launch  %6.2f TB/s\n", name, us, (double)NP * K * 2 / (us * 1e-6) / 1e12);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return 0;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const size_t bytes = (size_t)NP * K * 2;
    h16* W[3];
    for (int i = 0; i < 3; ++i) {
        CK(hipMalloc(&W[i], bytes));
        CK(hipMemset(W[i], 0, bytes));
    }
    float* out;
    CK(hipMalloc(&out, NP * 4 * 2));
    const int nblk = NP / 16;
    char name[128];
    for (int occ : {3, 4, 8}) {
        const size_t lds = occ >= 8 ? 0 : (160 * 1024) / occ - 1024;
        if (lds) {
            CK(hipFuncSetAttribute((const void*)gemv<0, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            CK(hipFuncSetAttribute((const void*)gemv<1, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            CK(hipFuncSetAttribute((const void*)gemv<1, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
            CK(hipFuncSetAttribute((const void*)gemv<0, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        }
        const int g1 = (nblk + 3) / 4, g2 = (nblk + 7) / 8;
        snprintf(name, sizeof name, "row-major  64 col/WG (%d WGs), %d WG/CU", g1, occ);
        if (time_graph(name, s, [&](int i) { gemv<0, 1><<<g1, 256, lds, s>>>(W[i], out); })) return 1;
        snprintf(name, sizeof name, "fragment   64 col/WG (%d WGs), %d WG/CU", g1, occ);
        if (time_graph(name, s, [&](int i) { gemv<1, 1><<<g1, 256, lds, s>>>(W[i], out); })) return 1;
        snprintf(name, sizeof name, "row-major 128 col/WG (%d WGs), %d WG/CU", g2, occ);
        if (time_graph(name, s, [&](int i) { gemv<0, 2><<<g2, 256, lds, s>>>(W[i], out); })) return 1;
        snprintf(name, sizeof name, "fragment  128 col/WG (%d WGs), %d WG/CU", g2, occ);
        if (time_graph(name, s, [&](int i) { gemv<1, 2><<<g2, 256, lds, s>>>(W[i], out); })) return 1;
    }
    const int64_t n4 = bytes / 16;
    for (int g : {768, 1024, 2048, 4096}) {
        snprintf(name, sizeof name, "copy-read float4 x8, %d WGs", g);
        if (time_graph(name, s, [&](int i) { copy_read<<<g, 256, 0, s>>>((const float4*)W[i], n4, out); })) return 1;
    }
    // MALL-resident reference: the same matrix every launch
    snprintf(name, sizeof name, "row-major 64 col/WG, one copy (MALL)");
    if (time_graph(name, s, [&](int) { gemv<0, 1><<<(nblk + 3) / 4, 256, 0, s>>>(W[0], out); })) return 1;
    snprintf(name, sizeof name, "fragment  64 col/WG, one copy (MALL)");
    if (time_graph(name, s, [&](int) { gemv<1, 1><<<(nblk + 3) / 4, 256, 0, s>>>(W[0], out); })) return 1;
    printf("done\n");
    return 0;
}
