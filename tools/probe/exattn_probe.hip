// Timing probe for the E-form cross-attention kernel (exattn.hip): the product kernel and
// variants with parts switched off (exattn_probe_kernel.inc, generated from the product
// kernel text: VAR bit 1 = no score MFMAs, 2 = no P.E MFMAs, 4 = no softmax phase and its
// two barriers), plus a plain streaming read of the same E bytes.  Large-v3-turbo shapes:
// W windows x 1500 x 1280 fp16.
// Regenerate the .inc: python3 tools/probe/make_exattn_probe.py
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/probe/exattn_probe tools/probe/exattn_probe.hip
#include "../../open-speech_amd/csrc/exattn.hip"

#include <cstdio>
#include <vector>

namespace osw {
namespace {
#include "exattn_probe_kernel.inc"

template <int NCH>
__global__ __launch_bounds__(512) void stream_kernel(const h16* __restrict__ E, int W, int T, int D, float* out) {
    const int w = blockIdx.x / NCH, c = blockIdx.x % NCH;
    const int per = (T + NCH - 1) / NCH;
    const int k0 = c * per, nk = min(T, k0 + per) - k0;
    const f32x4* p = (const f32x4*)(E + ((int64_t)w * T + k0) * D);
    const int n = nk * D / 8;
    float acc = 0.f;
    for (int i = threadIdx.x; i < n; i += 512 * 4) {
        f32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = (i + u * 512 < n) ? __builtin_nontemporal_load(p + i + u * 512) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += v[u][0] + v[u][1] + v[u][2] + v[u][3];
    }
    out[blockIdx.x * 512 + threadIdx.x] = acc;
}
}  // namespace
}  // namespace osw

using namespace osw;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 2; } } while (0)

template <class F>
static float time_us(F f, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    f(); f();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int i = 0; i < reps; ++i) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms * 1000.f / reps;
}

int main(int argc, char** argv) {
    const int W = argc > 1 ? atoi(argv[1]) : 64, T = 1500, D = 1280, H = 20, reps = 20;
    const int64_t ne = (int64_t)W * T * D, qlo = (int64_t)W * EX_HP * D;
    std::vector<h16> hE(ne), hq(2 * qlo);
    uint32_t x = 12345;
    for (auto& v : hE) { x = x * 1664525u + 1013904223u; v = (h16)(((x >> 9) & 1023) / 512.0f - 1.0f); }
    for (auto& v : hq) { x = x * 1664525u + 1013904223u; v = (h16)(((x >> 9) & 1023) / 4096.0f - 0.125f); }
    h16 *E, *qp, *pen; float *ws, *out; SelState* st;
    CK(hipMalloc(&E, ne * 2)); CK(hipMalloc(&qp, 2 * qlo * 2));
    CK(hipMalloc(&ws, (int64_t)W * 16 * H * (D + 8) * 4)); CK(hipMalloc(&pen, (int64_t)2 * W * H * D * 2));
    CK(hipMalloc(&st, W * sizeof(SelState))); CK(hipMalloc(&out, (size_t)W * 16 * 512 * 4));
    CK(hipMemset(st, 0, W * sizeof(SelState)));
    CK(hipMemcpy(E, hE.data(), ne * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(qp, hq.data(), 2 * qlo * 2, hipMemcpyHostToDevice));
    const double mb = ne * 2.0 / 1e6;
    const unsigned grid = (W + 7) / 8 * 8 * EX_CHUNKS;
    auto rep = [&](const char* name, float us) { printf("%-28s %8.2f us  %6.2f TB/s\n", name, us, mb / us); };
    rep("stream 4 chunks", time_us([&] { stream_kernel<4><<<W * 4, 512>>>(E, W, T, D, out); }, reps));
    rep("stream 8 chunks", time_us([&] { stream_kernel<8><<<W * 8, 512>>>(E, W, T, D, out); }, reps));
    rep("stream 16 chunks", time_us([&] { stream_kernel<16><<<W * 16, 512>>>(E, W, T, D, out); }, reps));
    rep("product exattn_kernel", time_us([&] { exattn_kernel<8, 160><<<grid, 512>>>(E, qp, qlo, W, T, H, ws, D + 8, st); }, reps));
#define PROBE(V, C, name) rep(name, time_us([&] { probe_kernel<8, 160, V, C><<<(W + 7) / 8 * 8 * C, 512>>>(E, qp, qlo, W, T, H, ws, D + 8, st); }, reps))
    PROBE(0, 4, "probe all, 4 chunks");
    PROBE(0, 8, "probe all, 8 chunks");
    PROBE(3, 4, "no MFMA");
    PROBE(4, 4, "no softmax");
    PROBE(7, 4, "staging + E reads");
    PROBE(15, 4, "staging only, 4 chunks");
    PROBE(15, 8, "staging only, 8 chunks");
    PROBE(15, 16, "staging only, 16 chunks");
    PROBE(7, 8, "staging + E reads, 8 chunks");
    PROBE(15 + 16, 4, "staging, no O stores");
    PROBE(15 + 32, 4, "staging, no q' loads");
    PROBE(15 + 48, 4, "staging, neither");
    PROBE(15 + 48, 8, "staging, neither, 8 chunks");
    PROBE(16, 4, "all, no O stores");
    PROBE(32, 4, "all, no q' loads");
    rep("launch_exattn (+ merge)", time_us([&] { launch_exattn(E, qp, qlo, W, T, D, ws, D + 8, pen, (int64_t)W * H * D, st, 0); }, reps));
    CK(hipDeviceSynchronize());
    printf("done\n");
    return 0;
}
