// Co-residency probe: can a small decoder-like workgroup start on a CU that runs an
// encoder-GEMM-like workgroup (512 threads, 128 KiB dynamic LDS, ~200 VGPRs, MFMA-heavy)?
// A "hog" kernel fills the chip on stream A for ~1 s; on stream B probe kernels with a
// given static LDS size (and VGPR footprint) run back to back; their mean time beside the
// hog vs alone tells whether they are placed beside it or wait for hog workgroups to end.
// build: hipcc --offload-arch=gfx950 -O3 tools/coresidency_probe.hip -o tools/coresidency_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// hog: every wave keeps 32 f32x4 MFMA accumulators (128 VGPRs) + operands live and runs
// `iters` MFMA rounds; LDS is touched so the dynamic allocation is real
__global__ __launch_bounds__(512, 1) void hog(float* out, int iters) {
    extern __shared__ float lds[];
    f32x4 acc[32];
    for (int i = 0; i < 32; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, (float)threadIdx.x};
    h16x8 a = (h16x8)(_Float16)1.0f, b = (h16x8)(_Float16)0.5f;
    lds[threadIdx.x] = 1.f;
    __syncthreads();
    a[0] = (_Float16)lds[(threadIdx.x + 1) & 511];
    for (int it = 0; it < iters; ++it) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 32; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[i], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    }
    float s = 0.f;
    for (int i = 0; i < 32; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    if (s == 12345.f) out[blockIdx.x] = s;
}

template <int LDSB>
__global__ __launch_bounds__(256) void probe(float* out) {
    __shared__ float buf[LDSB / 4 > 0 ? LDSB / 4 : 1];
    if (LDSB) {
        buf[threadIdx.x % (LDSB / 4 > 0 ? LDSB / 4 : 1)] = (float)threadIdx.x;
        __syncthreads();
        if (threadIdx.x == 0) out[blockIdx.x] = buf[(blockIdx.x * 7) % (LDSB / 4 > 0 ? LDSB / 4 : 1)];
    } else if (threadIdx.x == 0) {
        out[blockIdx.x] = 1.f;
    }
}

template <int LDSB>
float run_probe(hipStream_t s, float* out, int reps, int grid) {
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    CHK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) probe<LDSB><<<grid, 256, 0, s>>>(out);
    CHK(hipEventRecord(e1, s));
    CHK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    CHK(hipEventDestroy(e0));
    CHK(hipEventDestroy(e1));
    return 1000.f * ms / reps;
}

int main(int argc, char** argv) {
    const int hog_kb = argc > 1 ? atoi(argv[1]) : 128;
    float* out;
    CHK(hipMalloc(&out, 1 << 20));
    hipStream_t sa, sb;
    CHK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CHK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    CHK(hipFuncSetAttribute((const void*)hog, hipFuncAttributeMaxDynamicSharedMemorySize, hog_kb * 1024));
    // calibrate: one hog launch of 2048 workgroups
    hipEvent_t h0, h1;
    CHK(hipEventCreate(&h0));
    CHK(hipEventCreate(&h1));
    const int iters = 2000;
    CHK(hipEventRecord(h0, sa));
    hog<<<2048, 512, hog_kb * 1024, sa>>>(out, iters);
    CHK(hipEventRecord(h1, sa));
    CHK(hipEventSynchronize(h1));
    float hms = 0.f;
    CHK(hipEventElapsedTime(&hms, h0, h1));
    printf("hog: 2048 WGs x 512 threads, %d KiB dynamic LDS: %.2f ms (%.1f us per WG round)\n", hog_kb, hms,
           1000.f * hms / 8.f);
#define PROBE(L)                                                                                         \
    do {                                                                                                 \
        const float alone = run_probe<L>(sb, out, 200, 200);                                             \
        for (int k = 0; k < 8; ++k) hog<<<2048, 512, hog_kb * 1024, sa>>>(out, iters);                  \
        const float beside = run_probe<L>(sb, out, 200, 200);                                            \
        CHK(hipStreamSynchronize(sa));                                                                   \
        printf("probe LDS %6d B: alone %7.2f us  beside hog %8.2f us\n", L, alone, beside);           \
    } while (0)
    PROBE(0);
    PROBE(8192);
    PROBE(16384);
    PROBE(24576);
    PROBE(28672);
    PROBE(30720);
    PROBE(32768);
    CHK(hipDeviceSynchronize());
    printf("done\n");
    return 0;
}
