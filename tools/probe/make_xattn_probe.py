"""Generate tools/probe/xattn_probe_kernel.inc from the product dec_xattn_chunk_kernel:
the same text with VAR switches (bit 1: the K/V loads and one sum per lane only, 2: no q
reduction from the slabs, 4: no partial stores / ticket / merge)."""
import os

here = os.path.dirname(os.path.abspath(__file__))
src = open(os.path.join(here, "../../open-speech_amd/csrc/decode.hip")).read()
a = src.index("template <int NB>\n__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NB > 5 ? 4 : NB > 1 ? 5 : 1))) void dec_xattn_chunk_kernel(")
b = src.index("// Greedy rows when there are enough (window, head) pairs")
k = src[a:b].replace("void dec_xattn_chunk_kernel(", "void xprobe_kernel(").replace("template <int NB>", "template <int NB, int VAR>", 1)
reps = [
    ("""    // q of row r0 + k: fp16(bias + Σ split-K partials) / sqrt(64), the order of reduce_head""",
     """    if constexpr ((VAR & 1) != 0) {
        float s = 0.f;
#pragma unroll
        for (int u = 0; u < XU; ++u)
#pragma unroll
            for (int i = 0; i < 8; ++i) s += (float)kf[u][i] + (float)vf[u][i];
        if (s == 1234.5f) ws[tid] = s;
        return;
    }
    // q of row r0 + k: fp16(bias + Σ split-K partials) / sqrt(64), the order of reduce_head"""),
    ("""        for (; s + 4 < ks; s += 8) v += part[s * slab + off] + part[(s + 4) * slab + off];
        if (s < ks) v += part[s * slab + off];""",
     """        if constexpr ((VAR & 2) == 0) {
        for (; s + 4 < ks; s += 8) v += part[s * slab + off] + part[(s + 4) * slab + off];
        if (s < ks) v += part[s * slab + off];
        } else { v = 0.01f * lane; }"""),
    ("""    __syncthreads();
    __shared__ int last;
    if (wv == 0) {""",
     """    __syncthreads();
    if constexpr ((VAR & 4) != 0) {
        if (tid < NB * 64) out[(int64_t)p * 64 + tid] = (h16)(red[0][0][tid & 63] + rl[0][0]);
        return;
    }
    __shared__ int last;
    if (wv == 0) {"""),
]
for old, new in reps:
    assert k.count(old) == 1, old[:70]
    k = k.replace(old, new)
open(os.path.join(here, "xattn_probe_kernel.inc"), "w").write(k)
