// Audio ingest on the GPU, bit-exact with the reference's host numpy / scipy code:
//
//  * preprocess_stt_audio (/root/reference/src/audio/preprocessing.py:53-63):
//      mono = channel mean of int16 / 32768 (float32), rms over numpy's float32
//      pairwise summation, gain to -18 dBFS, clip, x 32767, truncating int16 cast.
//    ingest_sumsq_kernel reproduces numpy 2.x's np.add.reduce of a contiguous float32
//    vector: 8192-element blocks (the ufunc buffer), each by FLOAT_pairwise_sum
//    (leaves of <= 128 elements with 8 running sums, halving splits rounded down to
//    a multiple of 8; numpy/_core/src/umath/loops_utils.h.src), block sums added in
//    order on the host.  A full 8192 block is 64 leaves of 128 whose tree is the
//    lane butterfly of one wavefront (float addition is commutative, so a ^1 / ^2 /
//    ... exchange reproduces ((l0+l1)+(l2+l3))+... exactly).  The ragged tail block
//    is cut into its leaves on the host (ingest_tail_leaves), one lane per leaf.
//    ingest_gain_kernel: the per-sample float32 chain with every rounding explicit.
//  * resample_pcm16 (/root/reference/src/streaming.py:55-91): scipy 1.15
//    resample_poly(x, up, down, padtype="line") -> upfirdn in mode "line": one thread
//    per kept output sample, float32 multiply-then-add (never contracted to FMA: this
//    file is compiled under fp contract(off)) over the transposed, flipped polyphase taps in ascending
//    order from 0, out-of-range input samples from the line through x[0] and x[n-1];
//    then clip to the int16 range and truncate.
//
// Host side (buffers, tail-leaf tree, tap layout): osw.hip osw_ingest_*.
#include "common.h"

// every multiply and add below rounds on its own, like numpy's / scipy's C loops
// (hipcc otherwise contracts a*b+c into v_fma_f32, one rounding instead of two).  The
// operators are written out here: the pragma does not reach the bodies of header
// intrinsics such as __fmul_rn / __fadd_rn, whose operations stay contractible.
#pragma clang fp contract(off)

namespace osw {

namespace {
constexpr int PW_BLOCK = 8192;  // numpy ufunc buffer: elements per reduction inner loop
constexpr int PW_LEAF = 128;    // numpy PW_BLOCKSIZE

// float32 mono sample i of interleaved int16 PCM with `ch` channels (numpy: int16 ->
// float32, / 32768, then mean over the channel axis: sequential adds from channel 0,
// / ch as float32)
__device__ __forceinline__ float mono_sample(const int16_t* __restrict__ pcm, int64_t i, int ch) {
    const float k = 1.0f / 32768.0f;  // x / 32768 == x * 2^-15 exactly
    float s = (float)pcm[i * ch] * k;
    if (ch == 1) return s;
    for (int c = 1; c < ch; ++c) s = (s + (float)pcm[i * ch + c] * k);
    return (s / (float)ch);
}
__device__ __forceinline__ float sq(float x) { return (x * x); }

// numpy FLOAT_pairwise_sum of one leaf (n <= 128) of squares starting at sample i0
__device__ float leaf_sum(const int16_t* __restrict__ pcm, int64_t i0, int n, int ch) {
    if (n < 8) {
        float r = 0.f;
        for (int i = 0; i < n; ++i) r = (r + sq(mono_sample(pcm, i0 + i, ch)));
        return r;
    }
    float r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = sq(mono_sample(pcm, i0 + j, ch));
    const int m = n - n % 8;
    for (int i = 8; i < m; i += 8)
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = (r[j] + sq(mono_sample(pcm, i0 + i + j, ch)));
    float res = (((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7])));
    for (int i = m; i < n; ++i) res = (res + sq(mono_sample(pcm, i0 + i, ch)));
    return res;
}

// grid: n_full + 1 workgroups of 128 threads.  Workgroup b < n_full: the full block b
// (wave 0: leaf = lane, then the 6-level butterfly); the last workgroup: the tail's
// leaves, one per thread (<= 128 of them).
__global__ __launch_bounds__(128) void ingest_sumsq_kernel(const int16_t* __restrict__ pcm, int ch, int n_full,
                                                           const int2* __restrict__ tail_leaves, int n_tail_leaves,
                                                           float* __restrict__ block_sums,
                                                           float* __restrict__ tail_sums) {
    const int b = blockIdx.x, t = threadIdx.x;
    if (b < n_full) {
        if (t >= 64) return;
        float v = leaf_sum(pcm, (int64_t)b * PW_BLOCK + (int64_t)t * PW_LEAF, PW_LEAF, ch);
        v = (v + xor_lane<1>(v));
        v = (v + xor_lane<2>(v));
        v = (v + xor_lane<4>(v));
        v = (v + xor_lane<8>(v));
        v = (v + xor_lane<16>(v));
        v = (v + xor_lane<32>(v));
        if (t == 0) block_sums[b] = v;
        return;
    }
    if (t < n_tail_leaves) {
        const int2 lf = tail_leaves[t];
        tail_sums[t] = leaf_sum(pcm, (int64_t)n_full * PW_BLOCK + lf.x, lf.y, ch);
    }
}

// normalize_gain + float32_mono_to_wav_bytes per sample
__global__ __launch_bounds__(256) void ingest_gain_kernel(const int16_t* __restrict__ pcm, int64_t n, int ch,
                                                          int apply, float gain, int16_t* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        float a = mono_sample(pcm, i, ch);
        if (apply) a = fminf(fmaxf((a * gain), -1.0f), 1.0f);   // np.clip(audio * gain, -1, 1)
        a = fminf(fmaxf(a, -1.0f), 1.0f);                                  // np.clip(audio, -1, 1)
        out[i] = (int16_t)(a * 32767.0f);                          // astype(int16): truncation
    }
}

// upfirdn(h, x, up, down, mode="line") for the outputs [n_pre_remove, n_pre_remove + n_out)
__global__ __launch_bounds__(256) void ingest_resample_kernel(const int16_t* __restrict__ pcm, int64_t n_in,
                                                              const float* __restrict__ htf, int hpp, int up,
                                                              int down, int64_t n_pre_remove, int64_t n_out,
                                                              int16_t* __restrict__ out) {
    const int64_t y = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (y >= n_out) return;
    const float x0 = (float)pcm[0], xl = (float)pcm[n_in - 1];
    const float slope = ((xl - x0) / (float)(n_in - 1));
    const int64_t tt = (y + n_pre_remove) * down;
    const int64_t xi0 = tt / up - hpp + 1;
    const float* h = htf + (tt % up) * hpp;
    float acc = 0.f;
    for (int j = 0; j < hpp; ++j) {
        const int64_t i = xi0 + j;
        float v;
        if (i < 0) v = (x0 + ((float)i * slope));
        else if (i >= n_in) v = (xl + ((float)(i - n_in + 1) * slope));
        else v = (float)pcm[i];
        acc = (acc + (v * h[j]));
    }
    acc = fminf(fmaxf(acc, -32768.0f), 32767.0f);
    out[y] = (int16_t)acc;
}
}  // namespace

void launch_ingest_sumsq(const int16_t* pcm, int ch, int n_full, const int2* tail_leaves, int n_tail_leaves,
                         float* block_sums, float* tail_sums, hipStream_t s) {
    ingest_sumsq_kernel<<<n_full + 1, 128, 0, s>>>(pcm, ch, n_full, tail_leaves, n_tail_leaves, block_sums, tail_sums);
}

void launch_ingest_gain(const int16_t* pcm, int64_t n, int ch, int apply, float gain, int16_t* out, hipStream_t s) {
    const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    ingest_gain_kernel<<<blocks > 0 ? blocks : 1, 256, 0, s>>>(pcm, n, ch, apply, gain, out);
}

void launch_ingest_resample(const int16_t* pcm, int64_t n_in, const float* htf, int hpp, int up, int down,
                            int64_t n_pre_remove, int64_t n_out, int16_t* out, hipStream_t s) {
    ingest_resample_kernel<<<(unsigned)((n_out + 255) / 256), 256, 0, s>>>(pcm, n_in, htf, hpp, up, down, n_pre_remove,
                                                                        n_out, out);
}

}  // namespace osw
