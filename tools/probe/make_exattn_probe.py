"""Generate tools/probe/exattn_probe_kernel.inc from the product exattn_kernel: the same
text with VAR switches (bit 1: no score MFMAs, 2: no P.E MFMAs, 4: no softmax phase, 8: no E reads from LDS,
16: no O stores, 32: no q' loads;
NCH: key chunks per window)."""
import os

here = os.path.dirname(os.path.abspath(__file__))
src = open(os.path.join(here, "../../open-speech_amd/csrc/exattn.hip")).read()
a = src.index("// One (window, key chunk): partial (m, l, O[D]) per head over the chunk's keys.")
b = src.index("// (window, head): the EX_CHUNKS partials merged")
k = src[a:b].replace("void exattn_kernel(", "void probe_kernel(").replace("template <int NW, int JW>", "template <int NW, int JW, int VAR, int NCH>").replace("EX_CHUNKS", "NCH")
reps = [
    ("""                sp[ht] = __builtin_amdgcn_mfma_f32_16x16x32_f16(arow[s], qh[s][ht], sp[ht], 0, 0, 0);
                sp[ht] = __builtin_amdgcn_mfma_f32_16x16x32_f16(arow[s], ql[s][ht], sp[ht], 0, 0, 0);""",
     """                if constexpr (!(VAR & 1)) {
                sp[ht] = __builtin_amdgcn_mfma_f32_16x16x32_f16(arow[s], qh[s][ht], sp[ht], 0, 0, 0);
                sp[ht] = __builtin_amdgcn_mfma_f32_16x16x32_f16(arow[s], ql[s][ht], sp[ht], 0, 0, 0);
                } else { sp[ht] += arow[s][0]; }"""),
    ("""            o[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(acol[m], bh, o[m], 0, 0, 0);
            o[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(acol[m], bl, o[m], 0, 0, 0);""",
     """            if constexpr (!(VAR & 2)) {
            o[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(acol[m], bh, o[m], 0, 0, 0);
            o[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(acol[m], bl, o[m], 0, 0, 0);
            } else { o[m][0] += acol[m][0] + bh[0]; }"""),
    ("""        const h16* El = Es[wv][t % EX_NBUF];
#pragma unroll
        for (int s = 0; s < NS; ++s) arow[s]""", """        const h16* El = Es[wv][t % EX_NBUF];
        if constexpr (!(VAR & 8))
#pragma unroll
        for (int s = 0; s < NS; ++s) arow[s]"""),
    ("""        h16x4 tr[NM][2];
#pragma unroll
        for (int m = 0; m < NM; ++m)
#pragma unroll
            for (int r = 0; r < 2; ++r) {""", """        h16x4 tr[NM][2] = {};
        if constexpr (!(VAR & 8))
#pragma unroll
        for (int m = 0; m < NM; ++m)
#pragma unroll
            for (int r = 0; r < 2; ++r) {"""),
    ("""            scores(arow);
            ex_lds_barrier();
            softmax(t + 1);
            ex_lds_barrier();""",
     """            scores(arow);
            if constexpr (!(VAR & 4)) {
            ex_lds_barrier();
            softmax(t + 1);
            ex_lds_barrier();
            }"""),
]
reps += [
    ("""            qh[s][ht] = real ? *(const h16x8*)p : h16x8{};
            ql[s][ht] = real ? *(const h16x8*)(p + qlo) : h16x8{};""",
     """            qh[s][ht] = (real && !(VAR & 32)) ? *(const h16x8*)p : h16x8{};
            ql[s][ht] = (real && !(VAR & 32)) ? *(const h16x8*)(p + qlo) : h16x8{};"""),
    ("""    for (int idx = lane; idx < H * (JW / 4); idx += 64) {""",
     """    if (!(VAR & 16)) for (int idx = lane; idx < H * (JW / 4); idx += 64) {"""),
]
for old, new in reps:
    assert k.count(old) == 1, old[:60]
    k = k.replace(old, new)
open(os.path.join(here, "exattn_probe_kernel.inc"), "w").write(k)
