// Decoder-side state shared by decode.hip (kernels) and osw.hip (host pipeline).
#pragma once
#include "common.h"

namespace osw {

// Per decoder row (a window, or one beam hypothesis of a window).  Lives in device
// memory so a step needs no host round trip.
struct SelState {
    int n_sampled, last, penult, last_ts, done, lang;
    float sum_lp, nsp;  // greedy: Σ log-prob of the picks; beam: the hypothesis' cumulative score
    int plen;           // this row's prompt length (0: SelParams::prompt_len; decode sessions admit
                        // windows with different previous-text prefixes)
    int pad;
};

struct SelParams {
    int prompt_len;        // P: positions 0..P-1 are prompt (rows whose SelState::plen is 0)
    int sot_pos;           // position of <|startoftranscript|> in the prompt
    int lang_pos;          // prompt position holding the language token (-1 placeholder => detect)
    int max_length;
    int pstride;           // ints per row of the prompt buffer (>= every row's prompt length)
    int tail;              // prompt positions from <|startoftranscript|> to the end (3, or 4 with no-timestamps)
    int V, eot, no_speech, no_ts, tb, blank, first_lang, n_langs;
    int suppress_blank, with_ts, max_init_ts;
    int beam;              // hypotheses per window (1 = greedy)
    int num_hyp, max_cand; // beam stop rule: num_hypotheses, round(beam * patience)
    float length_penalty;
    float inv_temp;        // sampling (temperature > 0): 1 / temperature, else 0
    const unsigned long long* seed;  // device word: the draw seed (not in the graph key, so a new
                                     // seed per call replays the captured decode graph)
    const int* budget;     // per decoder row: force <|endoftext|> after this many sampled tokens (<= 0: none);
                           // nullptr: no budgets (osw_decode_opts::token_budget, length-controlled benches)
    int pos_row;           // 1: row r's step counter is pos[r] (row refill, sessions), 0: one shared counter
};

// the row's prompt length and <|startoftranscript|> position
__host__ __device__ __forceinline__ int row_plen(const SelParams& P, const SelState& s) {
    return s.plen > 0 ? s.plen : P.prompt_len;
}

// Per window in beam mode: finished-hypothesis bookkeeping (the best one's tokens
// are copied to a per-window buffer when it improves).
struct BeamWin {
    int n_hyp, best_len, done, pad;
    float best_norm, best_raw;
};

// Batch-1 greedy steps: the logits GEMM runs the token selection in its epilogue
// (gemm.hip, gemm_skinny_kernel<.., SEL>): every workgroup reduces its 64 columns to one
// slice record, the last to arrive merges them in workgroup order, finalises the row
// (select.h select_finalize) and advances the step counter -- no select launch.
struct SelFuse {
    SelParams P;
    const float* logits;  // this GEMM's output row (read back by the finaliser)
    int* pos;
    const unsigned* supmask;
    const int* prompt;
    SelState* st;
    int* cur_tok;
    int* tokens;
    int max_tokens;
    void* parts;   // one slice record per logits workgroup
    int* ticket;   // arrival counter (zero between launches)
};

constexpr int MAX_BEAM = 8;
constexpr int XPART = 72;     // floats per (decoder row, head, key chunk) cross-attention partial: m, l, pad, acc[64]
constexpr int XCHUNKS = 8;    // fixed key chunks per (window, head) in cross-attention
constexpr int SEL_SPLIT = 16;  // vocabulary slices per row in the selection kernels

void launch_session_rows(const int* pack, int k, int ps, int group, int pstride, int ctx, int* prompt, int* budget,
                         int* cur_tok, int* pos, SelState* st, int* anc, BeamWin* bwin, hipStream_t s);
void launch_refill_rows(const int* pack, int k, int P, int* prompt, int* budget, int* cur_tok, int* pos, SelState* st,
                        hipStream_t s);
void launch_select(const float* logits, int rows, int* pos, const SelParams& P, const int* prompt,
                   const unsigned* supmask, SelState* st, int* cur_tok, int* tokens, int max_tokens, void* sel_parts,
                   int* arrive, bool bump, void* cand, hipStream_t s);
// the last window's update advances *pos (arrive: a zeroed counter, left zeroed)
void launch_beam(const float* logits, int windows, int* pos, const SelParams& P, const unsigned* supmask,
                 SelState* st, const void* sel_parts, void* cand, int* seq, int* anc, int ctx, BeamWin* bw,
                 int* best_tok, int* cur_tok, int max_tokens, int* arrive, hipStream_t s);
int sel_parts_bytes();
int sel_fused_parts_bytes(int V);  // SelFuse::parts of the batch-1 logits GEMM (one record per 64 columns)
int beam_cand_bytes(int beam);
void launch_count_done(const SelState* st, int rows, int* out, hipStream_t s);

}  // namespace osw
