/*
 * osw.h — C ABI of libosw_hip.so, the MI355X (gfx950) Whisper transcription engine.
 *
 * This library is the drop-in for the arithmetic the reference delegates to
 * faster-whisper 1.2.1 / CTranslate2.  Each entry point names the reference
 * interface it replaces (paths under the reference repository):
 *
 *   osw_create / osw_set_weight / osw_init_weight_uniform / osw_finalize
 *       replace   WhisperModel(model_id, device, compute_type, download_root)
 *                 called at src/backends/faster_whisper.py:40-45 (load_model :29-50)
 *   osw_destroy
 *       replaces  del self._models[model_id]; gc; empty_cache   (unload_model :52-65)
 *   osw_transcribe_batch
 *       replaces  WhisperModel.transcribe(path, task, beam_size, temperature,
 *                 language, initial_prompt) + list(segments)     (:235-246),
 *                 for the first 30 s window of every clip; greedy, beam search
 *                 (beam_size > 1, the reference's default 5) or sampling
 *                 (temperature > 0, best_of rows), chosen per call by osw_decode_opts
 *   osw_log_mel / osw_encode_windows / osw_decode_windows
 *       the same work split by stage, as faster-whisper's generate_segments seek
 *       loop needs it (FeatureExtractor -> encode -> generate per 30 s window)
 *   osw_get_mel / osw_get_encoder_output / osw_encoder_layer_debug
 *       stage-level read-back used only by the parity tests
 *   osw_ingest_mean_square + osw_ingest_apply_gain
 *       replace   preprocess_stt_audio / normalize_gain (src/audio/preprocessing.py:35-63),
 *                 called at src/main.py:296-300; bit-identical output bytes
 *   osw_ingest_resample
 *       replaces  resample_pcm16 (src/streaming.py:55-91; scipy resample_poly,
 *                 padtype "line"), called at src/streaming.py:293-294; bit-identical
 *
 * Conventions: every call returns 0 (OSW_OK) or a negative code; the message of
 * the last failure on the calling thread is osw_last_error().  Host buffers are
 * caller-owned and only read/written during the call (the library copies them).
 * A context serialises its own calls (internal mutex); one context per device.
 * No torch types cross this boundary.
 *
 * Concurrency contract (the reference calls transcribe from several executor pools at
 * once, src/main.py:305, src/streaming.py:50-52, src/realtime/server.py:33-35, and loads
 * models on demand while serving, src/backends/faster_whisper.py:210-215):
 *   - any entry point may be called from any thread, on any context, at any time: calls
 *     on one context run one at a time; calls on different contexts (sibling lanes of
 *     one GPU, other GPUs, other models) run concurrently;
 *   - a context's decode steps are captured into hipGraphs on first use.  No entry point
 *     touches the legacy (null) stream: copies and memsets run on the context's own
 *     non-blocking stream.  Entry points that allocate, free, create or destroy streams
 *     (osw_create, osw_create_sibling, osw_destroy, osw_set_weight, osw_get_mel,
 *     osw_debug_gemm, a call whose input outgrows the resident buffers, the first ingest
 *     call on a device) wait for a capture in progress to end (one process-wide capture
 *     gate), so none of them can invalidate another context's capture;
 *   - the caller's own HIP / torch work in the same process must stay off the legacy
 *     stream while contexts are serving (e.g. run torch on a torch.cuda.Stream, which is
 *     non-blocking): HIP refuses legacy-stream work while any stream of the process
 *     captures, and the library cannot see it;
 *   - OSW_ECAPTURE reports a refused or invalidated stream capture: the context and the
 *     device remain usable, the call may be retried (it is not a device fault).
 */
#ifndef OSW_H
#define OSW_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OSW_OK 0
#define OSW_EINVAL (-22)
#define OSW_ENOMEM (-12)
#define OSW_EHIP (-100)
#define OSW_ESTATE (-101)
#define OSW_ECAPTURE (-102)

typedef struct osw_ctx osw_ctx;

typedef struct osw_dims {
    int32_t n_mels, n_audio_ctx, n_audio_state, n_audio_head, n_audio_layer;
    int32_t n_vocab, n_text_ctx, n_text_state, n_text_head, n_text_layer;
} osw_dims;

/* One 30 s decoding window: frames [seek, seek + segment_size) of clip `clip`'s
 * log-mel, zero padded to 3000 frames (faster-whisper pad_or_trim). */
typedef struct osw_window {
    int32_t clip;
    int32_t seek;
    int32_t segment_size;
} osw_window;

typedef struct osw_decode_opts {
    int32_t task_token;          /* <|transcribe|> or <|translate|> */
    int32_t language_token;      /* -1: detect from the <|startoftranscript|> logits */
    int32_t suppress_blank;      /* suppress " " and <|endoftext|> at the first sampled step */
    int32_t without_timestamps;  /* 0: timestamp rules on (faster-whisper default) */
    int32_t max_initial_timestamp_index; /* 50 = 1.0 s; -1 disables */
    int32_t max_length;          /* total positions (prompt + sampled), <= n_text_ctx */
    const int32_t* suppress_tokens; int32_t n_suppress;
    /* special token ids */
    int32_t eot, sot, sot_prev, no_speech, no_timestamps, timestamp_begin, blank;
    int32_t first_lang, n_langs;
    /* tokens placed BEFORE <|startoftranscript|> (e.g. <|startofprev|> + previous
     * text), n_windows * n_prefix ints, same length for every window of the call */
    const int32_t* prefix_tokens; int32_t n_prefix;
    /* optional per-window language tokens (n_windows ints; -1 = detect); NULL: use
     * language_token for every window */
    const int32_t* language_tokens;
    /* beam search (CTranslate2 BeamSearch semantics, as faster-whisper calls it):
     * beam_size <= 1 is greedy; windows * beam_size <= 5 * max_batch.  A caller
     * that sets beam_size > 1 must set length_penalty (0 = no length normalisation). */
    int32_t beam_size;           /* reference default 5 (src/backends/faster_whisper.py:237) */
    float patience;              /* <= 0 -> 1; stop once round(beam*patience) hypotheses finished */
    float length_penalty;        /* score / len**length_penalty ranks finished hypotheses */
    int32_t num_hypotheses;      /* <= 0 -> 1 */
    /* sampling = faster-whisper's temperature > 0 branch (beam 1, num_hypotheses = best_of,
     * sampling_topk 0): best_of decoder rows per window each draw every token from
     * softmax(logits / temperature) after the logits rules; the row with the best
     * sum_logprob / n_tokens**length_penalty is returned.  temperature <= 0: greedy or beam
     * search as above.  Replaces generate_with_fallback's sampling kwargs [upstream]. */
    float temperature;
    int32_t best_of;             /* <= 0 -> 1; windows * best_of <= 5 * max_batch */
    uint64_t seed;               /* draw seed (counter-hash Gumbel-max, reproducible) */
    /* length control (benches of realistic output lengths with random weights, which
     * never emit <|endoftext|> on their own): n_windows ints; greedy / sampling rows
     * emit <|endoftext|> once they have sampled token_budget[i] tokens, beam search
     * treats that step as the last one (<= 0: no limit).  NULL: off.  Not a reference
     * option. */
    const int32_t* token_budget;
} osw_decode_opts;

/* Caller-allocated outputs for n windows. */
typedef struct osw_window_result {
    int32_t* tokens;          /* [n][max_tokens]: sampled tokens (no prompt, no EOT) */
    int32_t max_tokens;
    int32_t* n_tokens;        /* [n] */
    float* sum_logprob;       /* [n]  includes the EOT step, as CTranslate2 scores do */
    float* no_speech_prob;    /* [n]  softmax(raw SOT logits)[no_speech] */
    int32_t* language;        /* [n]  language token used */
    float* logits_dump;       /* optional [n][dump_steps][n_vocab] raw logits of the first sampled steps */
    int32_t dump_steps;
} osw_window_result;

typedef struct osw_profile {
    double mel_ms, encoder_ms, crosskv_ms, decoder_ms, total_ms;
    int64_t decode_steps;           /* decoder steps launched in the last decode call */
    /* dominant-kernel accounting (HIP events around every launch of the class) */
    double enc_gemm_ms; int64_t enc_gemm_launches; double enc_gemm_flops;
    double enc_attn_ms; int64_t enc_attn_launches; double enc_attn_flops;
    double mel_kernel_ms; int64_t mel_kernel_launches; double mel_kernel_bytes;
    double xattn_ms; int64_t xattn_launches; double xattn_bytes;
} osw_profile;

const char* osw_version(void);
const char* osw_last_error(void);
int osw_device_count(int32_t* out);

int osw_create(const osw_dims* dims, int32_t device, int32_t max_batch, osw_ctx** out);
int osw_destroy(osw_ctx* ctx);
/* A second context on the parent's device that SHARES the parent's (finalized)
 * weights but owns its stream, workspaces and decode state.  Two contexts per GPU
 * driven from two host threads overlap one batch's MFMA-bound encoder with the
 * other's HBM/latency-bound decoder (the faster-whisper reference runs one
 * WhisperModel per process, src/backends/faster_whisper.py:40-45; this is the
 * batcher's per-GPU lane, not a reference entry point).  The weights stay alive
 * until the last context sharing them is destroyed; weight setters on a sibling
 * return OSW_EINVAL. */
int osw_create_sibling(osw_ctx* parent, int32_t max_batch, osw_ctx** out);

/* Sibling contexts serialise their encoders on the GPU (the encoder baton: one lane
 * encodes while the others decode); an encoder of fewer than `min_windows` windows skips
 * it, so small streaming encoders of sibling lanes run side by side.  Default 9
 * (OSW_BATON_MIN_WINDOWS); 0 = every encoder takes the baton.  Per context. */
int osw_set_encoder_baton_min(osw_ctx* ctx, int32_t min_windows);

/* Upload one canonical tensor (names and dtypes: open-speech_amd/weights.py). */
int osw_set_weight(osw_ctx* ctx, const char* name, const void* host, int64_t nbytes);
/* Read one tensor back as stored on the device (enc.conv1.w: the padded [De][3][C1]
 * layout).  For tests and checkpoint round trips. */
int osw_get_weight(osw_ctx* ctx, const char* name, void* host, int64_t nbytes);
/* Device-side counter-hash init: x[i] = (2u-1)*scale + offset, u from splitmix64. */
int osw_init_weight_uniform(osw_ctx* ctx, const char* name, uint64_t seed, int64_t stream,
                            float scale, float offset, int64_t zero_lo, int64_t zero_hi);
int osw_finalize(osw_ctx* ctx);   /* all tensors present? derive internal layouts */

/* PCM int16 of n_clips clips, clip i = pcm[offsets[i], offsets[i+1]).  When
 * pcm_on_device != 0, `pcm` is a device pointer on the context's device.
 * Computes the faster-whisper log-mel (padding 160, per-clip max clamp) and keeps it
 * resident; n_frames[i] receives the frame count of clip i. */
int osw_log_mel(osw_ctx* ctx, const int16_t* pcm, const int64_t* offsets, int32_t n_clips,
                int32_t pcm_on_device, int32_t* n_frames);
int osw_get_mel(osw_ctx* ctx, int32_t clip, float* out, int64_t out_floats);  /* [n_mels][n_frames] */

/* Encoder + cross-attention K/V for n windows of the resident log-mel. */
int osw_encode_windows(osw_ctx* ctx, const osw_window* windows, int32_t n);
int osw_get_encoder_output(osw_ctx* ctx, int32_t window, float* out, int64_t out_floats); /* [1500][D] */

/* Decode of the n windows last encoded, per `opts`: greedy (beam_size <= 1,
 * temperature <= 0), CTranslate2-style beam search (beam_size > 1; the reference calls
 * beam_size = 5, src/backends/faster_whisper.py:237) or sampling (temperature > 0,
 * best_of rows per window).  The prompt, logits rules and stop rules are the same in
 * all three modes. */
int osw_decode_windows(osw_ctx* ctx, int32_t n, const osw_decode_opts* opts, osw_window_result* res);

/* mel + encode + decode (greedy, beam search or sampling per `opts`, as
 * osw_decode_windows) of window 0 (seek 0, min(frames, 3000)) of every clip. */
int osw_transcribe_batch(osw_ctx* ctx, const int16_t* pcm, const int64_t* offsets, int32_t n_clips,
                         int32_t pcm_on_device, const osw_decode_opts* opts, osw_window_result* res);

/* Greedy transcription of window 0 of every clip (as osw_transcribe_batch) with row refill:
 * the decoder keeps max_batch rows, each with its own step counter, and a finished
 * window's row is refilled with the next queued clip (its window encoded straight into
 * that row's cross-K/V slot) once refill_min rows are free.  n_clips may exceed max_batch.
 * Each clip's result equals osw_transcribe_batch's.  Replaces the same per-file
 * WhisperModel.transcribe calls (src/backends/faster_whisper.py:235-246) when a caller has
 * many files queued; opts: temperature 0, beam_size 1, no prefix (OSW_EINVAL otherwise). */
int osw_transcribe_refill(osw_ctx* ctx, const int16_t* pcm, const int64_t* offsets, int32_t n_clips,
                          int32_t pcm_on_device, const osw_decode_opts* opts, osw_window_result* res,
                          int32_t refill_min);

/* ---- decode sessions: continuous batching of windows (greedy or beam search) ----
 * A session keeps max_batch window slots on the context (beam search: beam_size decoder
 * rows per slot, each with its own step counter and prompt).  Windows are queued with
 * osw_session_add and admitted into free slots between chunks of 8 decoder steps (their
 * encoder runs straight into the slot's cross-K/V); a finished window leaves its slot at
 * once.  So a window queued while others decode joins at the next chunk instead of
 * waiting for the longest window of a batch, and a caller can queue the next window of a
 * file (its previous-text prefix included) as soon as the previous one finished.  Each
 * window's result equals osw_decode_windows's for it alone: rows are independent in every
 * kernel.  Replaces the per-request WhisperModel.transcribe loops that the reference runs
 * from concurrent executor threads (src/main.py:305, src/streaming.py:366-375,
 * src/backends/faster_whisper.py:235-246) with one decoder batch per context.
 * opts: temperature 0 (greedy, or beam search with beam_size <= 5); its prefix_tokens,
 * language_tokens and token_budget are ignored (per window below).  While a session is
 * open the context's other decode entry points return OSW_EINVAL. */
typedef struct osw_session_window {
    int64_t tag;              /* the caller's id, returned with the result */
    int32_t seek;             /* first mel frame of the window in its clip */
    int32_t segment_size;     /* frames (<= 3000) */
    int32_t language_token;   /* -1: detect */
    int32_t token_budget;     /* length control (benches): <= 0 none */
    int32_t n_prefix;         /* previous-text prompt tokens before <|startoftranscript|> */
    const int32_t* prefix;    /* <|startofprev|> and the previous tokens, or NULL */
    /* >= 0: the caller's key of the window's clip.  The first window of a key brings the
     * clip's PCM; its log-mel is computed once and stays on the device, so later windows of
     * the same key pass no samples (offsets[i] == offsets[i+1]) and are staged from it,
     * until osw_session_release_clip(key) or osw_session_end.  < 0: the window's own PCM,
     * used for this window only. */
    int64_t clip;
} osw_session_window;
int osw_session_begin(osw_ctx* ctx, const osw_decode_opts* opts);
/* Queue n windows; window i reads clip pcm[offsets[i], offsets[i+1]) (host int16, copied). */
int osw_session_add(osw_ctx* ctx, const int16_t* pcm, const int64_t* offsets, int32_t n,
                    const osw_session_window* windows);
/* Admit queued windows into free slots (when at least min(refill_min, queued) slots are
 * free, or nothing decodes) and run up to max_chunks chunks of decoder steps, returning
 * after the first chunk in which windows finished (max_chunks 0: only admit, and wait for
 * the admitted windows' encoder).  Their results go to res[0 .. *n_done)
 * (res->tokens rows of res->max_tokens), their tags to tags_out; cap >= max_batch.
 * *n_active / *n_queued: windows decoding / waiting after the call. */
int osw_session_step(osw_ctx* ctx, int32_t max_chunks, int32_t refill_min, osw_window_result* res,
                     int64_t* tags_out, int32_t cap, int32_t* n_done, int32_t* n_active, int32_t* n_queued);
/* Frees the resident log-mel of clip `clip` (no queued window may still read it; windows
 * already admitted were staged and are unaffected). */
int osw_session_release_clip(osw_ctx* ctx, int64_t clip);
int osw_session_end(osw_ctx* ctx);

/* Parity helper: one encoder block on x [T][D] fp32 (host), result to y (host). */
int osw_encoder_layer_debug(osw_ctx* ctx, int32_t layer, const float* x, float* y, int32_t T);

/* Parity/timing helper: C[M][N] (fp32) = A[M][K] · W[N][K]ᵀ (fp16 host inputs) with GEMM
 * variant 0 = auto, 1 = 128x128 tile, 2 = 256x256 tile, 3 = skinny split-K (M <= 64);
 * runs `iters` times and stores the mean kernel time (ms, HIP events) in *ms. */
int osw_debug_gemm(osw_ctx* ctx, int32_t M, int32_t N, int32_t K, int32_t variant, const void* A, const void* W,
                   float* C, int32_t iters, float* ms);

/* Test hook for the concurrency contract: holds a stream capture open on the context's
 * stream for hold_ms (under the same locks as a decode-graph capture) and fails if it was
 * invalidated meanwhile.  Other threads' calls run during the hold. */
int osw_debug_hold_capture(osw_ctx* ctx, int32_t hold_ms);

/* 0 off; 1 per-stage HIP-event timers (decode steps stay in their hipGraph, so only
 * mel / encoder stages are timed); 2 also launches the decode steps eagerly so the
 * cross-attention timers see them.  Resets the counters. */
int osw_set_profiling(osw_ctx* ctx, int32_t enable);
int osw_get_profile(osw_ctx* ctx, osw_profile* out);
/* Device stream used by the context (hipStream_t as void*). */
void* osw_stream(osw_ctx* ctx);

/* ---- audio ingest (context-free: a per-device stream and scratch inside the library).
 * Host buffers in and out; the arithmetic runs on `device` and is bit-identical to the
 * reference's numpy / scipy code (csrc/ingest.hip).
 *
 * *out_mean = np.mean(np.square(mono)) in float32 with numpy's reduction order, where
 * mono = channel mean of pcm / 32768 (wav_bytes_to_float32_mono, preprocessing.py:9-20).
 * The caller derives the gain from it exactly as normalize_gain does (sqrt, log10,
 * 10 ** (dB / 20) on float32 scalars: preprocessing.py:36-41) and then calls
 * osw_ingest_apply_gain (apply_gain = 0 when normalize_gain returns early). */
int osw_ingest_mean_square(int32_t device, const int16_t* pcm, int64_t n_frames, int32_t channels, float* out_mean);
/* out[n_frames] = int16(clip(clip(mono * gain, -1, 1), -1, 1) * 32767) (truncating) */
int osw_ingest_apply_gain(int32_t device, const int16_t* pcm, int64_t n_frames, int32_t channels, int32_t apply_gain,
                          float gain, int16_t* out);
/* out[n_out] = resample_poly(pcm, up, down, padtype="line") clipped and truncated to
 * int16; h = the float32 filter resample_poly designs (firwin(2*10*max(up,down)+1,
 * 1/max(up,down), kaiser 5.0) cast to float32, times up), n_h odd; up/down already
 * divided by their gcd; n_in >= 2; n_out = ceil(n_in * up / down). */
int osw_ingest_resample(int32_t device, const int16_t* pcm, int64_t n_in, int32_t up, int32_t down, const float* h,
                        int32_t n_h, int16_t* out, int64_t n_out);

#ifdef __cplusplus
}
#endif
#endif /* OSW_H */
