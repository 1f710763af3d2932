// Minimal reproducer for the rocprofv3 --kernel-trace crash seen with concurrent
// decode-graph launches: T host threads, each with its own stream,
// capture a graph of K small kernel launches, instantiate it and replay it R times;
// with mode 1 one extra thread keeps capturing and instantiating NEW graphs meanwhile
// (what a lane does on the first call of a new decode-options key).  Mode 2 (VERDICT r4
// item 7, the state gpurun_out/r04_k/stream_probe_prof.txt:110-116 shows) adds a thread
// that launches kernels EAGERLY on its own stream, as osw_encode_windows does for an
// encoder below the baton threshold (a pageable H2D copy of the window table, ~300
// launches, an event record), while the capturing thread replays each freshly
// instantiated graph a few times.  No libosw code.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/graph_prof_repro tools/graph_prof_repro.hip -lpthread
// Run:   tools/graph_prof_repro [threads=3] [replays=300] [mode=1|2]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "%s: %s @%d\n", #x, hipGetErrorString(e_), __LINE__);     \
            std::exit(2);                                                                 \
        }                                                                                 \
    } while (0)

__global__ void step_kernel(float* x, int n, float a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x[i] = x[i] * a + 1.0f;
}

static hipGraphExec_t capture(hipStream_t s, float* buf, int n, int k) {
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < k; ++i) step_kernel<<<(n + 255) / 256, 256, 0, s>>>(buf, n, 0.5f + 0.01f * i);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphDestroy(g));
    return ge;
}

int main(int argc, char** argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 3;
    const int R = argc > 2 ? atoi(argv[2]) : 300;
    const int mode = argc > 3 ? atoi(argv[3]) : 1;
    const int n = 1 << 16, K = 32;
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([=] {
            hipStream_t s;
            float* buf;
            CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            CK(hipMalloc(&buf, n * sizeof(float)));
            CK(hipMemsetAsync(buf, 0, n * sizeof(float), s));
            hipGraphExec_t ge = capture(s, buf, n, K);
            for (int r = 0; r < R; ++r) {
                CK(hipGraphLaunch(ge, s));
                if (r % 16 == 15) CK(hipStreamSynchronize(s));
            }
            CK(hipStreamSynchronize(s));
            CK(hipGraphExecDestroy(ge));
            CK(hipFree(buf));
            CK(hipStreamDestroy(s));
        });
    if (mode == 2)
        th.emplace_back([=] {  // a sibling lane encoding eagerly beside the replays
            hipStream_t s;
            hipEvent_t ev;
            float* buf;
            int* win;
            CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            CK(hipMalloc(&buf, n * sizeof(float)));
            CK(hipMalloc(&win, 64 * sizeof(int)));
            std::vector<int> hw(64, 1);
            for (int r = 0; r < R / 4; ++r) {
                CK(hipMemcpyAsync(win, hw.data(), hw.size() * sizeof(int), hipMemcpyHostToDevice, s));
                for (int i = 0; i < 300; ++i) step_kernel<<<(n + 255) / 256, 256, 0, s>>>(buf, n, 0.5f);
                CK(hipEventRecord(ev, s));
                CK(hipEventSynchronize(ev));
            }
            CK(hipFree(win));
            CK(hipFree(buf));
            CK(hipEventDestroy(ev));
            CK(hipStreamDestroy(s));
        });
    if (mode >= 1)
        th.emplace_back([=] {  // a lane meeting new decode-options keys: capture after capture
            hipStream_t s;
            float* buf;
            CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            CK(hipMalloc(&buf, n * sizeof(float)));
            for (int r = 0; r < R / 4; ++r) {
                hipGraphExec_t ge = capture(s, buf, n, 8 + r % 8);
                for (int k = 0; k < (mode == 2 ? 4 : 1); ++k) CK(hipGraphLaunch(ge, s));
                CK(hipStreamSynchronize(s));
                CK(hipGraphExecDestroy(ge));
            }
            CK(hipFree(buf));
            CK(hipStreamDestroy(s));
        });
    for (auto& x : th) x.join();
    std::printf("graph_prof_repro: %d threads x %d replays (mode %d) done\n", T, R, mode);
    return 0;
}
