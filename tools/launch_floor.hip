// Per-launch floor of dependent kernels on one stream, replayed from a hipGraph (the
// decoder's execution mode): how much of the batch-1 decoder step (52 launches,
// ~350 us) is launch/boundary cost and how much is each kernel's own memory latency.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/launch_floor tools/launch_floor.hip
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

__global__ void k_empty(float* p) {
    if (p == nullptr) p[0] = 1.f;  // never taken
}
// one dependent global round trip: read what the previous launch wrote, write it back + 1
__global__ void k_chain(float* p) {
    if (threadIdx.x == 0 && blockIdx.x == 0) p[0] = p[0] + 1.f;
}
// every workgroup reads 64 KB (L2-resident) and writes one float
__global__ void k_read64k(const float4* __restrict__ src, float* dst) {
    float4 acc = {0, 0, 0, 0};
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) {
        float4 v = src[i];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    if (threadIdx.x == 0) dst[blockIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

template <typename F>
int time_graph(const char* name, hipStream_t s, int n, F&& launch) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < n; ++i) launch();
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(a, s));
    const int reps = 10;
    for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("%-44s %7.2f us per launch (graph of %d, %d replays)\n", name, ms * 1e3f / (reps * n), n, reps);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return 0;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    float* p;
    float4* src;
    CK(hipMalloc(&p, 1 << 20));
    CK(hipMalloc(&src, 1 << 20));
    CK(hipMemset(p, 0, 1 << 20));
    CK(hipMemset(src, 0, 1 << 20));
    const int n = 416;  // 8 decoder steps' worth of launches
    time_graph("empty, 1 WG x 64", s, n, [&] { k_empty<<<1, 64, 0, s>>>(p); });
    time_graph("empty, 256 WG x 256", s, n, [&] { k_empty<<<256, 256, 0, s>>>(p); });
    time_graph("empty, 2048 WG x 256", s, n, [&] { k_empty<<<2048, 256, 0, s>>>(p); });
    time_graph("dependent scalar chain, 1 WG", s, n, [&] { k_chain<<<1, 64, 0, s>>>(p); });
    time_graph("256 WG each read 64 KB (L2) + write", s, n, [&] { k_read64k<<<256, 256, 0, s>>>(src, p); });
    time_graph("1 WG x 1024 empty", s, n, [&] { k_empty<<<1, 1024, 0, s>>>(p); });
    printf("done\n");
    return 0;
}
