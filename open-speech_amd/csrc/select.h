// Whisper's token selection (greedy / sampling rules, slice statistics, row finaliser),
// shared by the select kernels (decode.hip) and the batch-1 logits GEMM that runs the
// selection in its epilogue (gemm.hip).  Included INSIDE each file's anonymous namespace
// (internal linkage per translation unit); needs common.h and decode.h.
#pragma once

// ---------------------------------------------------------------------------
// Greedy selection.  Per-window state lives in device memory so a step needs no
// host round trip.
struct ArgMax {
    float v;
    int i;
};
__device__ __forceinline__ ArgMax amax(ArgMax a, ArgMax b) {
    return (b.v > a.v || (b.v == a.v && b.i < a.i)) ? b : a;
}
__device__ __forceinline__ void lse_add(float& m, float& s, float x) {  // online log-sum-exp
    if (x == -INFINITY) return;
    if (x > m) {
        s = s * __expf(m - x) + 1.f;
        m = x;
    } else {
        s += __expf(x - m);
    }
}
__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
    if (m2 == -INFINITY) return;
    if (m == -INFINITY) { m = m2; s = s2; return; }
    if (m2 > m) { s = s * __expf(m - m2) + s2; m = m2; }
    else s += s2 * __expf(m2 - m);
}

// Per-window statistics over one vocabulary slice, with the logits rules applied
// on the fly (masked entries skipped):
//   m_all/s_all : online log-sum-exp over the kept entries
//   m_ts/s_ts   : the same over kept timestamp tokens
//   a_all/a_text/a_ts : argmax (lowest index on ties) over kept / kept text / kept timestamps
// At the <|startoftranscript|> step the slice stats are over the RAW logits and
// a_text is the argmax over the language tokens (language id + no-speech prob).
struct SelPart {
    float m_all, s_all, m_ts, s_ts;
    float v_all, v_text, v_ts;
    int i_all, i_text, i_ts;
};

enum { SEL_PROMPT = 0, SEL_SOT = 1, SEL_SAMPLE = 2, SEL_DONE = 3 };

__device__ __forceinline__ int sel_mode(const SelParams& P, int step, const SelState& s) {
    if (s.plen > 0) {  // a session row: its own prompt length
        if (step < s.plen - 1) return step == s.plen - P.tail ? SEL_SOT : SEL_PROMPT;
    } else if (step < P.prompt_len - 1) {
        return step == P.sot_pos ? SEL_SOT : SEL_PROMPT;
    }
    return s.done ? SEL_DONE : SEL_SAMPLE;
}

// The logits rules for one row at its current state (SuppressBlank, SuppressTokens,
// ApplyTimestampRules without the mass rule, which needs the slice statistics).
struct RowRules {
    int n, ts_block;
    bool last_ts, pen_ts;
};
__device__ __forceinline__ RowRules row_rules(const SelParams& P, const SelState& s) {
    RowRules R;
    R.n = s.n_sampled;
    R.last_ts = R.n >= 1 && s.last >= P.tb;
    R.pen_ts = R.n < 2 || s.penult >= P.tb;
    R.ts_block = P.tb;  // timestamps in [tb, ts_block) are forbidden (monotonicity)
    if (P.with_ts && s.last_ts > 0) R.ts_block = (R.last_ts && !R.pen_ts) ? s.last_ts : s.last_ts + 1;
    return R;
}
// word = supmask[v >> 5], the suppress-token bitmap word holding token v
__device__ __forceinline__ bool tok_masked_w(const SelParams& P, const RowRules& R, unsigned word, int v) {
    bool masked = (word >> (v & 31)) & 1u;
    if (P.suppress_blank && R.n == 0 && (v == P.blank || v == P.eot)) masked = true;
    if (P.with_ts) {
        if (v == P.no_ts) masked = true;
        if (R.last_ts) {
            if (R.pen_ts) { if (v >= P.tb) masked = true; }
            else { if (v < P.eot) masked = true; }
        }
        if (v >= P.tb && v < R.ts_block) masked = true;
        if (R.n == 0) {
            if (v < P.tb) masked = true;
            if (P.max_init_ts >= 0 && v > P.tb + P.max_init_ts) masked = true;
        }
    }
    return masked;
}

// Gumbel noise for sampling at temperature T: argmax_v(x_v / T + G(seed, row, step, v))
// is a draw from softmax(x / T) over the kept tokens (Gumbel-max).  G = -log(-log u),
// u from a splitmix64 hash of (seed, row, step, token) on 23 bits, so a draw does not
// depend on slice or lane order (oracle/decode.py restates it bit for bit).
__device__ __forceinline__ float gumbel_noise(unsigned long long seed, int row, int step, int v) {
    unsigned long long z = seed + 0x9E3779B97F4A7C15ull * (unsigned long long)(row + 1) +
                           0xD1B54A32D192ED03ull * (unsigned long long)(step + 1) +
                           0x94D049BB133111EBull * (unsigned long long)(v + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    const float u = ((float)(unsigned)(z >> 41) + 0.5f) * (1.0f / 8388608.0f);
    return -logf(-logf(u));
}

// Slice partials are published with device-scope stores (they write through the
// XCD's L2) and read back with device-scope loads by the row's finaliser, which may
// run on another XCD.
__device__ __forceinline__ void store_part(SelPart* dst, const SelPart& r) {
    float* f = (float*)dst;
    const float* v = (const float*)&r;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(SelPart) / 4); ++i)
        __hip_atomic_store(f + i, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ SelPart load_part(const SelPart* src) {
    SelPart r;
    float* v = (float*)&r;
    const float* f = (const float*)src;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(SelPart) / 4); ++i)
        v[i] = __hip_atomic_load(f + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return r;
}

// grid (B, SEL_SPLIT), 256 threads: one vocabulary slice of one row
template <bool SAMPLE>
__device__ __forceinline__ void select_partial_body(const float* __restrict__ logits, const SelParams& P, int step,
                                                    const unsigned* __restrict__ supmask,
                                                    const SelState* __restrict__ st, SelPart* __restrict__ parts) {
    const int b = blockIdx.x, sl = blockIdx.y, tid = threadIdx.x;
    const SelState s = st[b];
    const int mode = sel_mode(P, step, s);
    if (mode == SEL_PROMPT || mode == SEL_DONE) return;
    const float* x = logits + (int64_t)b * P.V;
    const int per = (P.V + SEL_SPLIT - 1) / SEL_SPLIT;
    const int lo = sl * per, hi = min(P.V, lo + per);
    const RowRules R = row_rules(P, s);
    float m_all = -INFINITY, s_all = 0.f, m_ts = -INFINITY, s_ts = 0.f;
    ArgMax a_all{-INFINITY, 0x7fffffff}, a_text{-INFINITY, 0x7fffffff}, a_ts{-INFINITY, 0x7fffffff};
    const unsigned long long seed = SAMPLE ? *P.seed : 0ull;
    // the thread's entries v = lo + tid + 256 i in order, their logits and suppress words
    // loaded 8 at a time (clamped addresses) before any is used: one memory round trip per
    // 8 entries instead of one per entry (batch 1: 18 -> 8 us per step)
    constexpr int SB = 8;
    for (int v0 = lo + tid; v0 < hi; v0 += 256 * SB) {
        float xs[SB];
        unsigned ws[SB];
#pragma unroll
        for (int j = 0; j < SB; ++j) {
            const int vv = min(v0 + 256 * j, hi - 1);
            xs[j] = x[vv];
            ws[j] = supmask[vv >> 5];
        }
#pragma unroll
        for (int j = 0; j < SB; ++j) {
            const int v = v0 + 256 * j;
            if (v >= hi) break;
            const float xv = xs[j];
            if (mode == SEL_SOT) {
                lse_add(m_all, s_all, xv);
                if (v >= P.first_lang && v < P.first_lang + P.n_langs) a_text = amax(a_text, ArgMax{xv, v});
                continue;
            }
            if (tok_masked_w(P, R, ws[j], v)) continue;
            lse_add(m_all, s_all, xv);
            // sampling: a_all / a_ts pick the Gumbel-perturbed maximum; a_text stays the plain
            // maximum (the timestamp-mass rule compares against it)
            const float key = SAMPLE ? xv * P.inv_temp + gumbel_noise(seed, b, step, v) : xv;
            a_all = amax(a_all, ArgMax{key, v});
            if (v >= P.tb) {
                lse_add(m_ts, s_ts, xv);
                a_ts = amax(a_ts, ArgMax{key, v});
            } else {
                a_text = amax(a_text, ArgMax{xv, v});
            }
        }
    }
    auto merge = [&](auto o) {
        constexpr int O = decltype(o)::value;
        lse_merge(m_all, s_all, xor_lane<O>(m_all), xor_lane<O>(s_all));
        lse_merge(m_ts, s_ts, xor_lane<O>(m_ts), xor_lane<O>(s_ts));
        a_all = amax(a_all, ArgMax{xor_lane<O>(a_all.v), xor_lane<O>(a_all.i)});
        a_text = amax(a_text, ArgMax{xor_lane<O>(a_text.v), xor_lane<O>(a_text.i)});
        a_ts = amax(a_ts, ArgMax{xor_lane<O>(a_ts.v), xor_lane<O>(a_ts.i)});
    };
    merge(IC<32>{}), merge(IC<16>{}), merge(IC<8>{}), merge(IC<4>{}), merge(IC<2>{}), merge(IC<1>{});
    __shared__ SelPart wp[4];
    const int w = tid >> 6;
    if ((tid & 63) == 0) wp[w] = SelPart{m_all, s_all, m_ts, s_ts, a_all.v, a_text.v, a_ts.v, a_all.i, a_text.i, a_ts.i};
    __syncthreads();
    if (tid == 0) {
        SelPart r = wp[0];
        for (int i = 1; i < 4; ++i) {
            const SelPart& q = wp[i];
            lse_merge(r.m_all, r.s_all, q.m_all, q.s_all);
            lse_merge(r.m_ts, r.s_ts, q.m_ts, q.s_ts);
            ArgMax A = amax(ArgMax{r.v_all, r.i_all}, ArgMax{q.v_all, q.i_all});
            ArgMax X = amax(ArgMax{r.v_text, r.i_text}, ArgMax{q.v_text, q.i_text});
            ArgMax T = amax(ArgMax{r.v_ts, r.i_ts}, ArgMax{q.v_ts, q.i_ts});
            r.v_all = A.v; r.i_all = A.i; r.v_text = X.v; r.i_text = X.i; r.v_ts = T.v; r.i_ts = T.i;
        }
        store_part(parts + b * SEL_SPLIT + sl, r);
    }
}

// DEVICE: the slices were written by other workgroups of the same launch (device-scope
// loads); otherwise by an earlier launch (plain loads).
template <bool DEVICE>
__device__ __forceinline__ SelPart combine_parts(const SelPart* __restrict__ parts) {
    SelPart r = DEVICE ? load_part(parts) : parts[0];
    // partly unrolled: fully unrolled, the 15 parts' loads were hoisted together and the
    // select kernel held 112 VGPRs for this one-thread tail
#pragma unroll 4
    for (int i = 1; i < SEL_SPLIT; ++i) {
        const SelPart q = DEVICE ? load_part(parts + i) : parts[i];
        lse_merge(r.m_all, r.s_all, q.m_all, q.s_all);
        lse_merge(r.m_ts, r.s_ts, q.m_ts, q.s_ts);
        ArgMax A = amax(ArgMax{r.v_all, r.i_all}, ArgMax{q.v_all, q.i_all});
        ArgMax X = amax(ArgMax{r.v_text, r.i_text}, ArgMax{q.v_text, q.i_text});
        ArgMax T = amax(ArgMax{r.v_ts, r.i_ts}, ArgMax{q.v_ts, q.i_ts});
        r.v_all = A.v; r.i_all = A.i; r.v_text = X.v; r.i_text = X.i; r.v_ts = T.v; r.i_ts = T.i;
    }
    return r;
}

// grid B, 64 threads: combine the slices in fixed order, apply the timestamp-mass
// rule, pick the token, update the window state.
// getr() returns the row's combined slice statistics (called only in the modes that use them).
// DEVLOAD: the logits were stored by other workgroups of the running launch (the fused
// batch-1 selection), so the few entries read back here use device-scope loads.
template <bool DEVLOAD = false, class GetR>
__device__ __forceinline__ void select_finalize(const float* __restrict__ logits, const SelParams& P, int step,
                                                const int* __restrict__ prompt, GetR getr,
                                                SelState* __restrict__ st, int* __restrict__ cur_tok,
                                                int* __restrict__ tokens, int max_tokens, int b) {
    auto lg = [&](int v) -> float {
        const float* p = logits + (int64_t)b * P.V + v;
        if constexpr (DEVLOAD) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return *p;
    };
    SelState s = st[b];
    const int mode = sel_mode(P, step, s);
    if (mode == SEL_PROMPT) {
        const int next = prompt[b * P.pstride + step + 1];
        cur_tok[b] = next < 0 ? s.lang : next;
        return;
    }
    if (mode == SEL_DONE) {
        cur_tok[b] = P.eot;
        return;
    }
    if (mode == SEL_SAMPLE && P.beam > 1) return;  // beam rows: beam_topk / beam_update
    const SelPart r = getr();
    const float lse_all = r.m_all + __logf(r.s_all);
    if (mode == SEL_SOT) {
        s.nsp = __expf(lg(P.no_speech) - lse_all);
        int next = prompt[b * P.pstride + step + 1];
        if (next < 0) {
            next = r.i_text;  // language detection: argmax over language tokens
            // no language won (NaN logits: a NaN never beats the {-inf, INT_MAX} seed of
            // amax): keep a valid token in the prompt and end the row, as beam_update does
            if (next < P.first_lang || next >= P.first_lang + P.n_langs) {
                next = P.first_lang;
                s.done = 1;
            }
        }
        s.lang = next;
        st[b] = s;
        cur_tok[b] = next;
        return;
    }
    const int n = s.n_sampled;
    int next = r.i_all;
    float lse = lse_all;
    if (P.with_ts) {
        const float lse_ts = r.m_ts == -INFINITY ? -INFINITY : r.m_ts + __logf(r.s_ts);
        if (lse_ts - lse_all > r.v_text - lse_all) {  // timestamp mass wins: text suppressed
            next = r.i_ts;
            lse = lse_ts;
        }
    }
    // no candidate won (an all-NaN row keeps the amax seed's INT_MAX): the row ends with
    // <|endoftext|> like beam_update's INT_MAX candidates, and nothing indexes with the id
    const bool none = (unsigned)next >= (unsigned)P.V;
    if (none) next = P.eot;
    // log-prob of the pick under the rule-masked, untempered distribution (what openai /
    // faster-whisper accumulate); sampling keys are perturbed, so read the logit back
    float lp = none ? lg(P.eot) - lse_all
                    : (P.inv_temp > 0.f ? lg(next) : (next == r.i_all ? r.v_all : r.v_ts)) - lse;
    if (P.budget && P.budget[b] > 0 && n >= P.budget[b]) {  // length control: the row ends here
        next = P.eot;
        lp = lg(P.eot) - lse_all;
    }
    s.sum_lp += lp;
    if (next == P.eot) {
        s.done = 1;
    } else {
        if (n < max_tokens) tokens[(int64_t)b * max_tokens + n] = next;
        s.n_sampled = n + 1;
        s.penult = s.last;
        s.last = next;
        if (next >= P.tb) s.last_ts = next;
        if (row_plen(P, s) + s.n_sampled >= P.max_length) s.done = 1;
    }
    st[b] = s;
    cur_tok[b] = next;
}

__device__ __forceinline__ void select_final_row(const float* __restrict__ logits, const SelParams& P, int step,
                                                 const int* __restrict__ prompt, const SelPart* __restrict__ parts,
                                                 SelState* __restrict__ st, int* __restrict__ cur_tok,
                                                 int* __restrict__ tokens, int max_tokens) {
    // this row's slices, staged in LDS
    select_finalize(logits, P, step, prompt, [&] { return combine_parts<false>(parts); }, st, cur_tok, tokens,
                    max_tokens, blockIdx.x);
}

