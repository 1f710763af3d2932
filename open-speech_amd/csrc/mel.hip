// Log-mel front end (faster-whisper FeatureExtractor semantics) on gfx950.
//
//   x = pcm/32768, zero-padded by 160 samples; frame t = centred (reflect) 400-sample
//   periodic-Hann window at hop 160; |rfft|^2 (201 bins); slaney mel bank; log10
//   clamp 1e-10; per-CLIP max (all frames) for the (max-8) clamp.
//
// Kernel 1 (mel_logmel_kernel): one workgroup = 16 frames of one clip.  The
// frames' 2800 samples are loaded once (coalesced int16) into LDS; the 400-point
// DFT is factored 400 = 16 x 25 (Cooley-Tukey, n = 25 n1 + n2, k = k1 + 16 k2):
// 25 real 16-point DFTs (9 outputs by conjugate symmetry) + twiddle, then 201
// 25-point DFTs, all from an LDS twiddle table computed in double on the host.
// The sparse slaney filters (each mel touches a contiguous bin range) give the
// mel energies; log10 values are written TIME-major [clip][t][n_mels] (512 B
// contiguous per frame) and the block max goes to one atomicMax per clip.
//
// Kernel 2 (mel_window_kernel): normalises ((max(v, gmax-8)+4)/4) a 3000-frame
// window [seek, seek+segment) into the fp16 conv1 operand X1[w][1+t][c] (zero
// rows at t=-1 and t=3000, zero pad past the segment = faster-whisper pad_or_trim).
#include "common.h"

namespace osw {

namespace {
constexpr int FPB = 16;          // frames per block (stage 2 maps FPB x 16 onto the 256 threads)
constexpr int NFFT = 400, HOP = 160, NBIN = 201;
constexpr int SPAN = HOP * (FPB - 1) + NFFT;  // 2800 samples

// w16^j = w400^(25 j) and w25^j = w400^(16 j), the host table's float values as
// constants (indices are compile-time after unrolling: immediates, no LDS reads)
constexpr float W16R[16] = {1.0f, 0.9238795042037964f, 0.7071067690849304f, 0.3826834261417389f, 6.123234262925839e-17f, -0.3826834261417389f, -0.7071067690849304f, -0.9238795042037964f, -1.0f, -0.9238795042037964f, -0.7071067690849304f, -0.3826834261417389f, -1.8369701465288538e-16f, 0.3826834261417389f, 0.7071067690849304f, 0.9238795042037964f};
constexpr float W16I[16] = {-0.0f, -0.3826834261417389f, -0.7071067690849304f, -0.9238795042037964f, -1.0f, -0.9238795042037964f, -0.7071067690849304f, -0.3826834261417389f, -1.2246468525851679e-16f, 0.3826834261417389f, 0.7071067690849304f, 0.9238795042037964f, 1.0f, 0.9238795042037964f, 0.7071067690849304f, 0.3826834261417389f};
constexpr float W25R[25] = {1.0f, 0.9685831665992737f, 0.8763066530227661f, 0.728968620300293f, 0.5358268022537231f, 0.30901700258255005f, 0.06279052048921585f, -0.187381312251091f, -0.4257792830467224f, -0.6374239921569824f, -0.80901700258255f, -0.9297764897346497f, -0.9921147227287292f, -0.9921147227287292f, -0.9297764897346497f, -0.80901700258255f, -0.6374239921569824f, -0.4257792830467224f, -0.187381312251091f, 0.06279052048921585f, 0.30901700258255005f, 0.5358268022537231f, 0.728968620300293f, 0.8763066530227661f, 0.9685831665992737f};
constexpr float W25I[25] = {-0.0f, -0.24868988990783691f, -0.4817536771297455f, -0.6845471262931824f, -0.8443279266357422f, -0.9510565400123596f, -0.9980267286300659f, -0.9822872281074524f, -0.9048270583152771f, -0.7705132365226746f, -0.5877852439880371f, -0.3681245446205139f, -0.12533323466777802f, 0.12533323466777802f, 0.3681245446205139f, 0.5877852439880371f, 0.7705132365226746f, 0.9048270583152771f, 0.9822872281074524f, 0.9980267286300659f, 0.9510565400123596f, 0.8443279266357422f, 0.6845471262931824f, 0.4817536771297455f, 0.24868988990783691f};

__device__ __forceinline__ int64_t reflect_idx(int64_t j, int64_t L) {
    if (L <= 1) return 0;
    const int64_t P = 2 * (L - 1);
    j %= P;
    if (j < 0) j += P;
    return j < L ? j : P - j;
}

__global__ __launch_bounds__(256) void mel_logmel_kernel(
    const int16_t* __restrict__ pcm, const int64_t* __restrict__ offsets, const int64_t* __restrict__ mel_off,
    const int* __restrict__ n_frames, const float2* __restrict__ tw400, const float* __restrict__ hann,
    const int* __restrict__ flo, const int* __restrict__ fcnt, const int* __restrict__ foff,
    const float* __restrict__ fw, int n_mels, float* __restrict__ logmel, int* __restrict__ clip_max) {
    __shared__ float xs[SPAN];
    __shared__ float2 tw[NFFT];
    __shared__ float win[NFFT];
    __shared__ float2 Z[FPB][25][16];
    __shared__ float P[FPB][NBIN + 3];
    __shared__ float red[8];

    const int clip = blockIdx.y;
    const int t0 = blockIdx.x * FPB;
    const int nf = n_frames[clip];
    if (t0 >= nf) return;
    const int tid = threadIdx.x;
    const int64_t base = offsets[clip];
    const int64_t N = offsets[clip + 1] - base;
    const int64_t L = N + HOP;  // padded length (padding = 160)

    for (int i = tid; i < NFFT; i += 256) {
        tw[i] = tw400[i];
        win[i] = hann[i];
    }
    const int64_t j0 = (int64_t)t0 * HOP - NFFT / 2;
    if (j0 >= 0 && j0 + SPAN <= N) {  // interior block: no reflection, no padding
        for (int i = tid; i < SPAN; i += 256) xs[i] = (float)pcm[base + j0 + i] * (1.0f / 32768.0f);
    } else {
        for (int i = tid; i < SPAN; i += 256) {
            const int64_t jj = reflect_idx(j0 + i, L);
            xs[i] = jj < N ? (float)pcm[base + jj] * (1.0f / 32768.0f) : 0.0f;
        }
    }
    __syncthreads();

    // stage 1: for (frame f, n2): Y[k1] = sum_n1 xw[25 n1 + n2] w16^(n1 k1), then * w400^(n2 k1)
    for (int task = tid; task < FPB * 25; task += 256) {
        const int f = task / 25, n2 = task % 25;
        float v[16];
#pragma unroll
        for (int n1 = 0; n1 < 16; ++n1) {
            const int n = 25 * n1 + n2;
            v[n1] = xs[f * HOP + n] * win[n];
        }
        float2 Y[9];
#pragma unroll
        for (int k1 = 0; k1 < 9; ++k1) {
            float re = 0.f, im = 0.f;
#pragma unroll
            for (int n1 = 0; n1 < 16; ++n1) {
                re = fmaf(v[n1], W16R[(n1 * k1) & 15], re);  // w16^(n1 k1)
                im = fmaf(v[n1], W16I[(n1 * k1) & 15], im);
            }
            Y[k1] = make_float2(re, im);
        }
#pragma unroll
        for (int k1 = 0; k1 < 16; ++k1) {
            const float2 y = k1 < 9 ? Y[k1] : make_float2(Y[16 - k1].x, -Y[16 - k1].y);
            const float2 w = tw[n2 * k1];  // n2*k1 <= 360
            Z[f][n2][k1] = make_float2(y.x * w.x - y.y * w.y, y.x * w.y + y.y * w.x);
        }
    }
    __syncthreads();

    // stage 2: X[k1 + 16 k2] = sum_n2 Z[n2][k1] w25^(n2 k2); power spectrum.  One
    // thread per (frame, k1): its 25 Z values are read once and feed all k2 (<= 13).
    {
        const int f = tid >> 4, k1 = tid & 15;  // FPB * 16 == 256 threads
        float2 z[25];
#pragma unroll
        for (int n2 = 0; n2 < 25; ++n2) z[n2] = Z[f][n2][k1];
#pragma unroll
        for (int k2 = 0; k2 < 13; ++k2) {
            const int k = k1 + 16 * k2;
            if (k < NBIN) {
                float re = 0.f, im = 0.f;
#pragma unroll
                for (int n2 = 0; n2 < 25; ++n2) {
                    const float wr = W25R[(n2 * k2) % 25], wi = W25I[(n2 * k2) % 25];
                    re += z[n2].x * wr - z[n2].y * wi;
                    im += z[n2].x * wi + z[n2].y * wr;
                }
                P[f][k] = re * re + im * im;
            }
        }
    }
    __syncthreads();

    // stage 3: mel, log10; time-major store; block max.  Thread = (mel m, half of the
    // frames): the filter's weights are read once for 8 frames.
    float lmax = -INFINITY;
    for (int task = tid; task < 2 * n_mels; task += 256) {
        const int m = task % n_mels, f0 = (task / n_mels) * (FPB / 2);
        const int lo = flo[m], cnt = fcnt[m], off = foff[m];
        float s[FPB / 2];
#pragma unroll
        for (int j = 0; j < FPB / 2; ++j) s[j] = 0.f;
        for (int i = 0; i < cnt; ++i) {
            const float wgt = fw[off + i];
#pragma unroll
            for (int j = 0; j < FPB / 2; ++j) s[j] = fmaf(wgt, P[f0 + j][lo + i], s[j]);
        }
#pragma unroll
        for (int j = 0; j < FPB / 2; ++j) {
            const int t = t0 + f0 + j;
            if (t >= nf) break;
            const float lg = log10f(fmaxf(s[j], 1e-10f));
            logmel[mel_off[clip] + (int64_t)t * n_mels + m] = lg;
            lmax = fmaxf(lmax, lg);
        }
    }
    lmax = wave_max(lmax);
    if ((tid & 63) == 0) red[tid >> 6] = lmax;
    __syncthreads();
    if (tid == 0) {
        float m = red[0];
        for (int i = 1; i < 4; ++i) m = fmaxf(m, red[i]);
        atomicMax(&clip_max[clip], float_to_ordered(m));
    }
}

__global__ void mel_max_init_kernel(int* clip_max, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) clip_max[i] = float_to_ordered(-INFINITY);
}

// X1[w][r][c], r in [0, 3002), c in [0, C1): fp16 normalised window, zero borders/pad
__global__ __launch_bounds__(256) void mel_window_kernel(
    const float* __restrict__ logmel, const int64_t* __restrict__ mel_off, const int* __restrict__ n_frames,
    const int* __restrict__ clip_max, const int* __restrict__ win_clip, const int* __restrict__ win_seek,
    const int* __restrict__ win_size, int n_mels, int C1, h16* __restrict__ X1) {
    const int w = blockIdx.y;
    const int clip = win_clip[w], seek = win_seek[w];
    const int seg = min(win_size[w], n_frames[clip] - seek);
    const float gmax = ordered_to_float(clip_max[clip]);
    const float floor_v = gmax - 8.0f;
    const int64_t rows_total = 3002;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < rows_total * C1;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int r = (int)(idx / C1), c = (int)(idx % C1);
        const int t = r - 1;
        float v = 0.f;
        if (t >= 0 && t < 3000 && t < seg && c < n_mels) {
            const float x = logmel[mel_off[clip] + (int64_t)(seek + t) * n_mels + c];
            v = (fmaxf(x, floor_v) + 4.0f) * 0.25f;
        }
        X1[(int64_t)w * rows_total * C1 + idx] = (h16)v;
    }
}

// normalised fp32 mel, mel-major [n_mels][nf] (parity read-back)
__global__ void mel_normalize_kernel(const float* __restrict__ logmel, int64_t off, int nf, int n_mels,
                                     const int* __restrict__ clip_max, int clip, float* __restrict__ out) {
    const float floor_v = ordered_to_float(clip_max[clip]) - 8.0f;
    const int64_t total = (int64_t)nf * n_mels;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int m = (int)(i / nf), t = (int)(i % nf);
        out[i] = (fmaxf(logmel[off + (int64_t)t * n_mels + m], floor_v) + 4.0f) * 0.25f;
    }
}
}  // namespace

void launch_mel(const int16_t* pcm, const int64_t* offsets, const int64_t* mel_off, const int* n_frames,
                int n_clips, int max_frames, const float2* tw400, const float* hann, const int* flo,
                const int* fcnt, const int* foff, const float* fw, int n_mels, float* logmel, int* clip_max,
                hipStream_t s) {
    mel_max_init_kernel<<<(n_clips + 255) / 256, 256, 0, s>>>(clip_max, n_clips);
    dim3 grid((max_frames + FPB - 1) / FPB, n_clips);
    mel_logmel_kernel<<<grid, 256, 0, s>>>(pcm, offsets, mel_off, n_frames, tw400, hann, flo, fcnt, foff, fw,
                                           n_mels, logmel, clip_max);
}

void launch_mel_window(const float* logmel, const int64_t* mel_off, const int* n_frames, const int* clip_max,
                       const int* win_clip, const int* win_seek, const int* win_size, int n_windows, int n_mels,
                       int C1, h16* X1, hipStream_t s) {
    dim3 grid(256, n_windows);
    mel_window_kernel<<<grid, 256, 0, s>>>(logmel, mel_off, n_frames, clip_max, win_clip, win_seek, win_size,
                                           n_mels, C1, X1);
}

void launch_mel_normalize(const float* logmel, int64_t off, int nf, int n_mels, const int* clip_max, int clip,
                          float* out, hipStream_t s) {
    mel_normalize_kernel<<<512, 256, 0, s>>>(logmel, off, nf, n_mels, clip_max, clip, out);
}

}  // namespace osw
