// libosw_hip.so runtime: context, weights, resident buffers, encoder / decoder
// pipelines and the C ABI of include/osw.h.
//
// One context = one device, one HIP stream, buffers sized for `max_batch` windows
// at creation (nothing is allocated in the per-call hot path except when a call
// brings more PCM / mel than any earlier call).  Calls on one context are
// serialised by a mutex; independent contexts (one per GPU) run concurrently.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <pthread.h>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/osw.h"
#include "common.h"
#include "decode.h"
#include "resln.h"

namespace osw {
// launchers from the other translation units
void launch_mel(const int16_t*, const int64_t*, const int64_t*, const int*, int, int, const float2*, const float*,
                const int*, const int*, const int*, const float*, int, float*, int*, hipStream_t);
void launch_mel_window(const float*, const int64_t*, const int*, const int*, const int*, const int*, const int*, int,
                       int, int, h16*, hipStream_t);
void launch_mel_normalize(const float*, int64_t, int, int, const int*, int, float*, hipStream_t);
void launch_enc_attn(const h16*, h16*, int, int, int, hipStream_t);
void launch_init_uniform(void*, bool, int64_t, uint64_t, float, float, int64_t, int64_t, hipStream_t);
uint64_t hash_stream_key(uint64_t, int64_t);
void launch_dec_self_attn(const float*, int, const float*, h16*, h16*, const int*, int, int, int, h16*, int64_t,
                          const int*, int, const SelState*, hipStream_t, int pos_row = 0);
void launch_dec_cross_attn(const float*, int, const float*, const h16*, const h16*, int, int, int, int, h16*, int64_t,
                           float*, int*, const SelState*, hipStream_t);
void launch_dec_resid_ln(const float*, int, int, int, const float*, float*, const float*, const float*, h16*, int64_t,
                         const h16*, const float*, const int*, const int*, int, int, hipStream_t, int pos_row = 0);
void launch_dec_reduce_gelu(const float*, int, int, int, const float*, h16*, int64_t, hipStream_t);
void launch_ingest_sumsq(const int16_t*, int, int, const int2*, int, float*, float*, hipStream_t);
void launch_ingest_gain(const int16_t*, int64_t, int, int, float, int16_t*, hipStream_t);
void launch_ingest_resample(const int16_t*, int64_t, const float*, int, int, int, int64_t, int64_t, int16_t*,
                            hipStream_t);
}  // namespace osw

using namespace osw;

namespace {
thread_local std::string g_err;

struct OswError : std::runtime_error {
    int code;
    OswError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// Stream-capture errors are refusals of an operation, not device faults: the context and
// the GPU stay usable, so they get their own code (OSW_ECAPTURE) and the serving layer does
// not fail the GPU over on them (runner.py).
inline int hip_code(hipError_t e) {
    switch (e) {
        case hipErrorStreamCaptureUnsupported:
        case hipErrorStreamCaptureInvalidated:
        case hipErrorStreamCaptureMerge:
        case hipErrorStreamCaptureUnmatched:
        case hipErrorStreamCaptureUnjoined:
        case hipErrorStreamCaptureIsolation:
        case hipErrorStreamCaptureImplicit:
        case hipErrorCapturedEvent:
        case hipErrorStreamCaptureWrongThread:
            return OSW_ECAPTURE;
        default:
            return OSW_EHIP;
    }
}
#define HIPCHK(x)                                                                                  \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess)                                                                      \
            throw OswError(hip_code(e_), std::string(#x) + ": " + hipGetErrorString(e_) + " @" +   \
                                             std::to_string(__LINE__));                            \
    } while (0)
#define REQUIRE(c, msg) \
    do {                \
        if (!(c)) throw OswError(OSW_EINVAL, msg); \
    } while (0)

template <typename F>
int guard(F&& f) {
    try {
        f();
        return OSW_OK;
    } catch (const OswError& e) {
        g_err = e.what();
        return e.code;
    } catch (const std::bad_alloc&) {
        g_err = "out of host memory";
        return OSW_ENOMEM;
    } catch (const std::exception& e) {
        g_err = e.what();
        return OSW_ESTATE;
    }
}

struct Tensor {
    void* ptr = nullptr;
    int64_t numel = 0;
    bool f16 = true;
    bool set = false;
    // a decoder matrix the skinny GEMM streams: N x K, with a fragment-major copy in the
    // tensor "<name>.frag" (GemmArgs::Wf), repacked whenever the matrix is written
    int frag_n = 0, frag_k = 0;
};

// The capture gate (one per process).  While a stream is being captured into a hipGraph,
// HIP refuses every operation that would make the legacy (null) stream depend on it
// ("operation would make the legacy stream depend on a capturing blocking stream") and
// invalidates the capture; its capture-status check spans every stream of the process, so
// a synchronous hipMemcpy / hipMemset, hipMalloc / hipFree, hipDeviceSynchronize or stream
// creation on one lane's thread breaks a sibling lane's capture (GPUTEST_r05).  So:
//   * a decode graph is captured only while holding this gate (decode_graph);
//   * every allocation, free, stream / pinned-buffer creation or destruction and every
//     implicitly synchronising call takes it too (dalloc / dfree, osw_create,
//     osw_create_sibling, osw_destroy, osw_set_weight, osw_get_mel, osw_debug_gemm, ingest);
//   * everything else a call does runs on the context's own non-blocking stream
//     (hipMemcpyAsync / hipMemsetAsync + hipStreamSynchronize), never on the legacy stream.
// Recursive: osw_create holds it across setup_workspace's dalloc calls.  Lock order: a
// context's mu, then the encoder baton's mu, then this gate; nothing is locked under it.
std::recursive_mutex& capture_gate() {
    static std::recursive_mutex m;
    return m;
}
using GateLock = std::lock_guard<std::recursive_mutex>;

template <typename T>
T* dalloc(size_t n, std::vector<void*>& owned) {
    GateLock gate_(capture_gate());
    void* p = nullptr;
    if (n == 0) n = 1;
    hipError_t e = hipMalloc(&p, n * sizeof(T));
    if (e != hipSuccess) throw OswError(OSW_ENOMEM, "hipMalloc " + std::to_string(n * sizeof(T)) + " B failed");
    owned.push_back(p);
    return (T*)p;
}

// Frees a buffer dalloc'd into `owned` (implicitly synchronises the device; growth only).
template <typename T>
void dfree(T*& p, std::vector<void*>& owned) {
    if (!p) return;
    for (auto it = owned.begin(); it != owned.end(); ++it)
        if (*it == (void*)p) {
            owned.erase(it);
            break;
        }
    GateLock gate_(capture_gate());
    (void)hipFree(p);
    p = nullptr;
}

// Makes `device` current for one C-ABI call and restores the caller's device after it:
// a host thread that calls into the library and then issues its own HIP / torch work
// stays on the GPU it was on.
struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(int device) {
        HIPCHK(hipGetDevice(&prev));
        if (prev != device) HIPCHK(hipSetDevice(device));
    }
    ~DeviceScope() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
    DeviceScope(const DeviceScope&) = delete;
    DeviceScope& operator=(const DeviceScope&) = delete;
};

struct EventPair {
    hipEvent_t a, b;
    int cls;
    double work;
};

// Encoder baton, shared by a context and its siblings (the lanes of one GPU): each
// lane's encoder waits on the GPU for the previous lane's encoder to finish.  The
// encoder is MFMA-bound and fills every CU, so two encoders side by side only
// time-slice; lanes started together would otherwise stay in lock-step (all encoders,
// then all decoders) and never overlap an encoder with the others' HBM/latency-bound
// decoders, which is what the lanes are for.
struct EncBaton {
    std::mutex mu;
    hipEvent_t ev = nullptr;
    bool recorded = false;
    // calls in flight over the contexts sharing this baton (LaneCall): with more than one,
    // the encoder GEMMs leave a quarter of the CUs to the other lanes (GemmArgs::share_cus)
    std::atomic<int> in_call{0};
    ~EncBaton() {
        if (ev) (void)hipEventDestroy(ev);
    }
};
}  // namespace

struct osw_ctx {
    std::mutex mu;
    int device = 0;
    hipStream_t stream = nullptr;
    osw_dims d{};
    int B = 0;    // max windows per call
    int R = 0;    // decoder row capacity (windows x beam hypotheses)
    int C1 = 0;   // conv1 input channels padded to a multiple of 64
    std::vector<void*> owned;
    std::map<std::string, Tensor> w;
    std::shared_ptr<void> arena;  // weight arena, shared with sibling contexts (osw_create_sibling)
    bool sibling = false;         // weights belong to another context: read-only here
    bool finalized = false;
    std::shared_ptr<EncBaton> baton;  // shared with sibling contexts; null: encoders not serialised
    int baton_min = 9;                // encoders of fewer windows skip the baton (osw_set_encoder_baton_min)
    bool share_cus = false;           // this call's encoder GEMMs leave CUs to sibling lanes
    // OSW_ENC_PRIO=1: the encoder runs on its own low-priority stream, the decoder on a
    // high-priority `stream` (measured slower: the default is one stream per lane)
    hipStream_t enc_stream = nullptr;
    hipEvent_t enc_in = nullptr, enc_out = nullptr;

    // mel constants
    float2* tw400 = nullptr;
    float* hann = nullptr;
    int *flo = nullptr, *fcnt = nullptr, *foff = nullptr;
    float* fw = nullptr;
    // resident mel
    int16_t* pcm = nullptr;
    size_t pcm_cap = 0;
    int64_t* offsets = nullptr;
    int64_t* mel_off_d = nullptr;
    int* nframes_d = nullptr;
    int* clip_max = nullptr;
    int clips_cap = 0;
    float* logmel = nullptr;
    size_t logmel_cap = 0;
    int n_clips = 0;
    std::vector<int> nframes;
    std::vector<int64_t> mel_off;

    // encoder workspace
    int* win = nullptr;  // [3][B]
    h16 *X1 = nullptr, *H1 = nullptr, *Xn = nullptr, *QKV = nullptr, *O = nullptr, *Hf = nullptr, *E = nullptr,
        *XKV = nullptr;
    float* X = nullptr;
    int n_encoded = 0;
    bool row_pos = false;             // decode_refill / sessions: per-row step counters (pos[row])
    int kv_rows = 0;                  // sessions: self-K/V cache rows per layer (0: the step's row count)
    int xkv_windows = 0;              // sessions: cross-K/V windows per layer (0: the step's windows)
    struct Session* sess = nullptr;   // an open decode session (osw_session_*)
    struct ClipStore* cstore = nullptr;  // decode sessions' resident clip log-mels (created on first use)
    int* slot_d = nullptr;            // encode into slots: window -> decoder row
    int* refill_pack = nullptr;       // decode_refill: rows to admit {row, budget, prompt}

    // decoder workspace.  xdn / dattn / dh (the GEMM operands) are hi/lo fp16 pairs:
    // the lo halves sit R rows after the hi halves (lo_off below)
    float* xd = nullptr;
    float* xd2 = nullptr;      // second residual buffer of the fused small-batch step (ping-pong)
    h16 *xdn = nullptr, *dqkv = nullptr, *dattn = nullptr, *dq = nullptr, *dh = nullptr, *kc = nullptr, *vc = nullptr;
    float* logits = nullptr;
    int *cur_tok = nullptr, *pos = nullptr, *tokens = nullptr, *prompt = nullptr, *done = nullptr;
    unsigned* supmask = nullptr;
    SelState* sel = nullptr;   // per decoder row
    void* selp = nullptr;      // per-row vocabulary-slice partial stats
    void* selp1 = nullptr;     // batch-1 fused selection: one record per logits workgroup
    int* anc = nullptr;        // beam: [R][ctx] row whose cache slot holds position p of this hypothesis
    int* btok = nullptr;       // beam: [B][ctx] best finished hypothesis per window
    BeamWin* bwin = nullptr;   // beam: [B]
    void* bcand = nullptr;     // beam: [R][SEL_SPLIT][2 lists][2*MAX_BEAM] candidates (beam_slice_body)
    int* done_host = nullptr;  // pinned
    float* part = nullptr;     // split-K partial slabs of the decoder GEMMs
    float* part2 = nullptr;    // second slab buffer of the fused small-batch step (<= PRO_ROWS rows)
    float* xws = nullptr;      // cross-attention per-chunk partials [R][H][XCHUNKS][XPART]
    int* xticket = nullptr;    // cross-attention arrival tickets [B][H] (zero between launches)
    int* tail_ticket = nullptr; // split-K GEMM tails (ProArgs::tail_ticket)
    int* sel_arrive = nullptr; // select arrival counters: rows finalised + per-row slice tickets (zero between launches)
    int* budget = nullptr;     // per-row token budgets (osw_decode_opts::token_budget)
    unsigned long long* seed_d = nullptr;  // sampling seed of the current decode call
    int64_t part_floats = 0;

    // decode-step graphs (CH steps per replay), one per key (batch rows, prompt length,
    // decode options); a small LRU so a serving mix of batch sizes replays instead of
    // re-capturing (the streaming collator meets batches of 1..4 windows)
    std::map<std::vector<int64_t>, std::pair<hipGraphExec_t, uint64_t>> dgraphs;
    uint64_t dgraph_tick = 0;
    hipGraphExec_t dgraph = nullptr;
    bool capturing = false;
    bool prof_eager = false;  // profiling mode 2: decode steps launched eagerly so the per-kernel timers see them
    bool use_graph = true;

    // profiling
    bool prof = false;
    osw_profile pf{};
    std::vector<EventPair> evs;
    std::vector<hipEvent_t> ev_free;
};

namespace {
const int T_ENC = 1500;
const int N_FR = 3000;

// OSW_TRACE_GRAPH=1: one stderr line per decode-graph event (capture, instantiate, launch,
// LRU destroy) with the calling thread and context, to correlate host-side crashes of a
// tool that intercepts HIP (e.g. a profiler) with what the lanes were doing
void trace_graph(const osw_ctx* c, const char* what) {
    static const bool on = [] {
        const char* e = std::getenv("OSW_TRACE_GRAPH");
        return e && e[0] == '1';
    }();
    if (!on) return;
    std::fprintf(stderr, "[osw-graph] thread %zx ctx %p %s\n", (size_t)pthread_self(), (const void*)c, what);
    std::fflush(stderr);
}

hipEvent_t get_ev(osw_ctx* c) {
    if (!c->ev_free.empty()) {
        hipEvent_t e = c->ev_free.back();
        c->ev_free.pop_back();
        return e;
    }
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    return e;
}

// class ids for per-launch accounting
enum { CL_ENC_GEMM = 1, CL_ENC_ATTN = 2, CL_MEL = 3, CL_XATTN = 4, CL_STAGE_MEL = 10, CL_STAGE_ENC = 11,
       CL_STAGE_XKV = 12, CL_STAGE_DEC = 13 };

struct Timed {
    osw_ctx* c;
    EventPair p{};
    bool on;
    Timed(osw_ctx* c_, int cls, double work) : c(c_), on(c_->prof && !c_->capturing) {
        if (!on) return;
        p.a = get_ev(c);
        p.b = get_ev(c);
        p.cls = cls;
        p.work = work;
        HIPCHK(hipEventRecord(p.a, c->stream));
    }
    ~Timed() {
        if (!on) return;
        if (hipEventRecord(p.b, c->stream) == hipSuccess) c->evs.push_back(p);
    }
};

void resolve_events(osw_ctx* c) {
    if (c->evs.empty()) return;
    HIPCHK(hipStreamSynchronize(c->stream));
    for (auto& e : c->evs) {
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, e.a, e.b));
        osw_profile& p = c->pf;
        switch (e.cls) {
            case CL_ENC_GEMM: p.enc_gemm_ms += ms; p.enc_gemm_launches++; p.enc_gemm_flops += e.work; break;
            case CL_ENC_ATTN: p.enc_attn_ms += ms; p.enc_attn_launches++; p.enc_attn_flops += e.work; break;
            case CL_MEL: p.mel_kernel_ms += ms; p.mel_kernel_launches++; p.mel_kernel_bytes += e.work; break;
            case CL_XATTN: p.xattn_ms += ms; p.xattn_launches++; p.xattn_bytes += e.work; break;
            case CL_STAGE_MEL: p.mel_ms += ms; break;
            case CL_STAGE_ENC: p.encoder_ms += ms; break;
            case CL_STAGE_XKV: p.crosskv_ms += ms; break;
            case CL_STAGE_DEC: p.decoder_ms += ms; break;
        }
        c->ev_free.push_back(e.a);
        c->ev_free.push_back(e.b);
    }
    c->evs.clear();
}

// ---------------------------------------------------------------------------
void add_tensor(osw_ctx* c, const std::string& name, int64_t numel, bool f16) {
    Tensor t;
    t.numel = numel;
    t.f16 = f16;
    c->w[name] = t;
}

void build_weight_table(osw_ctx* c) {
    const osw_dims& d = c->d;
    const int64_t De = d.n_audio_state, Dd = d.n_text_state, L = d.n_text_layer;
    add_tensor(c, "enc.conv1.w", De * 3 * c->C1, true);  // stored padded [De][3][C1]
    add_tensor(c, "enc.conv1.b", De, false);
    add_tensor(c, "enc.conv2.w", De * 3 * De, true);
    add_tensor(c, "enc.conv2.b", De, false);
    add_tensor(c, "enc.pos", (int64_t)d.n_audio_ctx * De, false);
    for (int i = 0; i < d.n_audio_layer; ++i) {
        const std::string p = "enc.l" + std::to_string(i);
        add_tensor(c, p + ".ln1.g", De, false);
        add_tensor(c, p + ".ln1.b", De, false);
        add_tensor(c, p + ".qkv.w", 3 * De * De, true);
        add_tensor(c, p + ".qkv.b", 3 * De, false);
        add_tensor(c, p + ".o.w", De * De, true);
        add_tensor(c, p + ".o.b", De, false);
        add_tensor(c, p + ".ln2.g", De, false);
        add_tensor(c, p + ".ln2.b", De, false);
        add_tensor(c, p + ".fc1.w", 4 * De * De, true);
        add_tensor(c, p + ".fc1.b", 4 * De, false);
        add_tensor(c, p + ".fc2.w", 4 * De * De, true);
        add_tensor(c, p + ".fc2.b", De, false);
    }
    add_tensor(c, "enc.lnpost.g", De, false);
    add_tensor(c, "enc.lnpost.b", De, false);
    add_tensor(c, "dec.tok", (int64_t)d.n_vocab * Dd, true);
    add_tensor(c, "dec.pos", (int64_t)d.n_text_ctx * Dd, false);
    add_tensor(c, "dec.crosskv.w", L * 2 * Dd * De, true);
    add_tensor(c, "dec.crosskv.b", L * 2 * Dd, false);
    for (int i = 0; i < d.n_text_layer; ++i) {
        const std::string p = "dec.l" + std::to_string(i);
        add_tensor(c, p + ".ln1.g", Dd, false);
        add_tensor(c, p + ".ln1.b", Dd, false);
        add_tensor(c, p + ".qkv.w", 3 * Dd * Dd, true);
        add_tensor(c, p + ".qkv.b", 3 * Dd, false);
        add_tensor(c, p + ".o.w", Dd * Dd, true);
        add_tensor(c, p + ".o.b", Dd, false);
        add_tensor(c, p + ".ln2.g", Dd, false);
        add_tensor(c, p + ".ln2.b", Dd, false);
        add_tensor(c, p + ".xq.w", Dd * Dd, true);
        add_tensor(c, p + ".xq.b", Dd, false);
        add_tensor(c, p + ".xo.w", Dd * Dd, true);
        add_tensor(c, p + ".xo.b", Dd, false);
        add_tensor(c, p + ".ln3.g", Dd, false);
        add_tensor(c, p + ".ln3.b", Dd, false);
        add_tensor(c, p + ".fc1.w", 4 * Dd * Dd, true);
        add_tensor(c, p + ".fc1.b", 4 * Dd, false);
        add_tensor(c, p + ".fc2.w", 4 * Dd * Dd, true);
        add_tensor(c, p + ".fc2.b", Dd, false);
    }
    add_tensor(c, "dec.lnpost.g", Dd, false);
    add_tensor(c, "dec.lnpost.b", Dd, false);
    // fragment-major copies of what the skinny decoder GEMMs stream (+ 0.3 GB at turbo):
    // measured on the 133 MB logits matrix (tools/gemv_probe.hip), the 1-KB contiguous
    // fragment loads stream 5.2-5.4 TB/s against 3.9-4.2 TB/s for 16 rows x 64 B
    auto frag = [&](const std::string& n, int64_t N, int64_t K) {
        Tensor& t = c->w[n];
        t.frag_n = (int)N;
        t.frag_k = (int)K;
        add_tensor(c, n + ".frag", (N + 15) / 16 * 16 * K, true);
        c->w[n + ".frag"].set = true;  // derived: written by pack_frag
    };
    frag("dec.tok", d.n_vocab, Dd);
    for (int i = 0; i < d.n_text_layer; ++i) {
        const std::string p = "dec.l" + std::to_string(i);
        frag(p + ".qkv.w", 3 * Dd, Dd);
        frag(p + ".o.w", Dd, Dd);
        frag(p + ".xq.w", Dd, Dd);
        frag(p + ".xo.w", Dd, Dd);
        frag(p + ".fc1.w", 4 * Dd, Dd);
        frag(p + ".fc2.w", Dd, 4 * Dd);
    }

    // one arena, every tensor 256-B aligned
    size_t total = 0;
    for (auto& kv : c->w) total += ((size_t)kv.second.numel * (kv.second.f16 ? 2 : 4) + 255) & ~(size_t)255;
    void* ap = nullptr;
    GateLock gate_(capture_gate());
    if (hipMalloc(&ap, total) != hipSuccess)
        throw OswError(OSW_ENOMEM, "hipMalloc " + std::to_string(total) + " B (weights) failed");
    const int dev = c->device;
    c->arena = std::shared_ptr<void>(ap, [dev](void* p) {
        GateLock gate_(capture_gate());
        int prev = -1;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(dev);
        (void)hipFree(p);
        if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
    });
    char* arena = (char*)ap;
    HIPCHK(hipMemsetAsync(arena, 0, total, c->stream));
    size_t off = 0;
    for (auto& kv : c->w) {
        kv.second.ptr = arena + off;
        off += ((size_t)kv.second.numel * (kv.second.f16 ? 2 : 4) + 255) & ~(size_t)255;
    }
}

Tensor& W(osw_ctx* c, const std::string& n) {
    auto it = c->w.find(n);
    if (it == c->w.end()) throw OswError(OSW_EINVAL, "unknown tensor " + n);
    return it->second;
}
const h16* WH(osw_ctx* c, const std::string& n) { return (const h16*)W(c, n).ptr; }
const float* WF(osw_ctx* c, const std::string& n) { return (const float*)W(c, n).ptr; }
// the fragment-major copy of a decoder matrix (GemmArgs::Wf); OSW_NO_WFRAG=1: row-major (A/B)
const h16* WFR(osw_ctx* c, const std::string& n) {
    static const bool off = getenv("OSW_NO_WFRAG") != nullptr;
    if (off) return nullptr;
    auto it = c->w.find(n + ".frag");
    return it == c->w.end() ? nullptr : (const h16*)it->second.ptr;
}
// rewrite the fragment-major copy after the matrix was written (on the context's stream)
void pack_frag(osw_ctx* c, const std::string& n) {
    const Tensor& t = W(c, n);
    if (!t.frag_n) return;
    launch_frag_pack((const h16*)t.ptr, t.frag_k, t.frag_n, t.frag_k, (h16*)W(c, n + ".frag").ptr, c->stream);
    HIPCHK(hipGetLastError());
}

// --------------------------- mel constants ---------------------------------
double hz_to_mel(double f) {
    const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp, logstep = std::log(6.4) / 27.0;
    return f >= min_log_hz ? min_log_mel + std::log(f / min_log_hz) / logstep : f / f_sp;
}
double mel_to_hz(double m) {
    const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp, logstep = std::log(6.4) / 27.0;
    return m >= min_log_mel ? min_log_hz * std::exp(logstep * (m - min_log_mel)) : f_sp * m;
}

void setup_mel(osw_ctx* c) {
    const int n_mels = c->d.n_mels;
    std::vector<float2> tw(400);
    std::vector<float> hn(400);
    for (int j = 0; j < 400; ++j) {
        const double a = 2.0 * M_PI * j / 400.0;
        tw[j] = make_float2((float)std::cos(a), (float)-std::sin(a));
        hn[j] = (float)(0.5 - 0.5 * std::cos(a));
    }
    // slaney mel bank (librosa / faster-whisper get_mel_filters), double precision
    std::vector<double> mel_f(n_mels + 2);
    const double mmin = hz_to_mel(0.0), mmax = hz_to_mel(8000.0);
    for (int i = 0; i < n_mels + 2; ++i) mel_f[i] = mel_to_hz(mmin + (mmax - mmin) * i / (n_mels + 1));
    std::vector<int> lo(n_mels), cnt(n_mels), off(n_mels);
    std::vector<float> wts;
    for (int m = 0; m < n_mels; ++m) {
        const double enorm = 2.0 / (mel_f[m + 2] - mel_f[m]);
        int first = -1, last = -1;
        std::vector<float> row(201);
        for (int k = 0; k < 201; ++k) {
            const double f = k * 16000.0 / 400.0;
            const double lower = -(mel_f[m] - f) / (mel_f[m + 1] - mel_f[m]);
            const double upper = (mel_f[m + 2] - f) / (mel_f[m + 2] - mel_f[m + 1]);
            const double v = std::max(0.0, std::min(lower, upper)) * enorm;
            row[k] = (float)v;
            if (v > 0) {
                if (first < 0) first = k;
                last = k;
            }
        }
        if (first < 0) first = last = 0;
        lo[m] = first;
        cnt[m] = last - first + 1;
        off[m] = (int)wts.size();
        for (int k = first; k <= last; ++k) wts.push_back(row[k]);
    }
    // (the host vectors live until the copies are done: synchronised before returning)
    c->tw400 = dalloc<float2>(400, c->owned);
    c->hann = dalloc<float>(400, c->owned);
    c->flo = dalloc<int>(n_mels, c->owned);
    c->fcnt = dalloc<int>(n_mels, c->owned);
    c->foff = dalloc<int>(n_mels, c->owned);
    c->fw = dalloc<float>(wts.size(), c->owned);
    HIPCHK(hipMemcpyAsync(c->tw400, tw.data(), 400 * sizeof(float2), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->hann, hn.data(), 400 * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->flo, lo.data(), n_mels * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->fcnt, cnt.data(), n_mels * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->foff, off.data(), n_mels * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->fw, wts.data(), wts.size() * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
}

void setup_workspace(osw_ctx* c) {
    const osw_dims& d = c->d;
    const int64_t B = c->B, De = d.n_audio_state, Dd = d.n_text_state;
    const int64_t Me = B * T_ENC;
    auto& o = c->owned;
    c->win = dalloc<int>(3 * B, o);
    c->X1 = dalloc<h16>(B * 3002 * c->C1, o);
    c->H1 = dalloc<h16>(B * 3001 * De, o);
    HIPCHK(hipMemsetAsync(c->H1, 0, (size_t)B * 3001 * De * 2, c->stream));  // row 0 of every window stays zero
    c->X = dalloc<float>(Me * De, o);
    c->Xn = dalloc<h16>(Me * De, o);
    c->QKV = dalloc<h16>(3 * Me * De, o);
    c->O = dalloc<h16>(Me * De, o);
    c->Hf = dalloc<h16>(Me * 4 * De, o);
    c->E = dalloc<h16>(Me * De, o);
    c->XKV = dalloc<h16>((int64_t)d.n_text_layer * 2 * Me * Dd, o);
    const int64_t R = c->R;
    c->xd = dalloc<float>(R * Dd, o);
    c->xd2 = dalloc<float>(std::min<int64_t>(R, PRO_ROWS) * Dd, o);
    c->xdn = dalloc<h16>(2 * R * Dd, o);
    c->dqkv = dalloc<h16>(R * 3 * Dd, o);
    c->dattn = dalloc<h16>(2 * R * Dd, o);
    c->dq = dalloc<h16>(R * Dd, o);
    c->dh = dalloc<h16>(2 * R * 4 * Dd, o);
    const int64_t kvn = (int64_t)d.n_text_layer * R * d.n_text_ctx * Dd;
    c->kc = dalloc<h16>(kvn, o);
    c->vc = dalloc<h16>(kvn, o);
    c->logits = dalloc<float>(R * d.n_vocab, o);
    c->cur_tok = dalloc<int>(R, o);
    c->pos = dalloc<int>(R, o);  // [0]: the shared step counter; [row] in decode_refill
    c->slot_d = dalloc<int>(B, o);
    c->refill_pack = dalloc<int>(B * (3 + d.n_text_ctx), o);  // (sessions: {slot, plen, budget, prompt})
    c->tokens = dalloc<int>(R * d.n_text_ctx, o);
    c->prompt = dalloc<int>(R * d.n_text_ctx, o);
    c->done = dalloc<int>(1, o);
    c->supmask = dalloc<unsigned>((d.n_vocab + 31) / 32, o);
    c->sel = dalloc<SelState>(R, o);
    c->selp = dalloc<char>((size_t)R * sel_parts_bytes(), o);
    c->selp1 = dalloc<char>((size_t)sel_fused_parts_bytes(d.n_vocab), o);
    c->anc = dalloc<int>(R * d.n_text_ctx, o);
    c->btok = dalloc<int>(B * d.n_text_ctx, o);
    c->bwin = dalloc<BeamWin>(B, o);
    c->bcand = dalloc<char>((size_t)R * beam_cand_bytes(MAX_BEAM), o);
    c->xws = dalloc<float>(R * d.n_text_head * XCHUNKS * XPART, o);
    c->xticket = dalloc<int>(B * d.n_text_head, o);
    HIPCHK(hipMemsetAsync(c->xticket, 0, (size_t)B * d.n_text_head * sizeof(int), c->stream));
    c->budget = dalloc<int>(R, o);
    c->seed_d = dalloc<unsigned long long>(1, o);
    c->tail_ticket = dalloc<int>(4096, o);  // GEMM tails: [column blocks x row groups] (zero between launches)
    HIPCHK(hipMemsetAsync(c->tail_ticket, 0, 4096 * sizeof(int), c->stream));
    c->sel_arrive = dalloc<int>(1 + R, o);  // [0] rows finalised, [1 + row] slice tickets
    HIPCHK(hipMemsetAsync(c->sel_arrive, 0, (1 + (size_t)R) * sizeof(int), c->stream));
    {
        const int64_t shapes[][2] = {{3 * Dd, Dd}, {Dd, Dd}, {4 * Dd, Dd}, {Dd, 4 * Dd}, {d.n_vocab, Dd}};
        for (auto& nk : shapes)  // skinny split-K slabs: decoder projections at any row count
            c->part_floats = std::max<int64_t>(c->part_floats,
                                               skinny_ksplit((int)nk[0], (int)nk[1]) * nk[0] *
                                                   (nk[0] == d.n_vocab ? std::min<int64_t>(R, 64) : R));
        for (auto& nk : shapes)  // > 64 rows: split-K slabs of the tiled GEMM
            if (R > 64 && nk[0] != d.n_vocab)
                c->part_floats = std::max<int64_t>(c->part_floats,
                                                   (int64_t)tiled_ksplit((int)R, (int)nk[0], (int)nk[1]) * R * nk[0]);
        c->part = dalloc<float>(c->part_floats, o);
        int64_t p2 = 0;
        for (auto& nk : shapes)
            if (nk[0] != d.n_vocab) p2 = std::max<int64_t>(p2, (int64_t)skinny_ksplit((int)nk[0], (int)nk[1]) * nk[0]);
        c->part2 = dalloc<float>(p2 * std::min<int64_t>(R, GELU_ROWS), o);
    }
    GateLock gate_(capture_gate());
    HIPCHK(hipHostMalloc((void**)&c->done_host, sizeof(int), 0));
}

// A transcription call in flight on a context: counted on the baton its siblings share,
// and decides whether this call's encoder GEMMs share the CUs (another lane is busy too)
struct LaneCall {
    osw_ctx* c;
    explicit LaneCall(osw_ctx* c_) : c(c_) {
        c->share_cus = c->baton && c->baton->in_call.fetch_add(1) > 0;
    }
    ~LaneCall() {
        if (c->baton) c->baton->in_call.fetch_sub(1);
    }
};

// ------------------------------ GEMM helper ---------------------------------
GemmArgs gemm_plain(const h16* A, int64_t lda, const h16* Wt, const float* bias, int M, int N, int K, void* C,
                    int64_t ldc, int epi) {
    GemmArgs g{};
    g.A = A; g.lda = lda; g.a_grp_rows = M; g.a_grp_stride = 0;
    g.W = Wt; g.ldw = K; g.bias = bias; g.M = M; g.N = N; g.K = K;
    g.C = C; g.ldc = ldc; g.c_grp_rows = M; g.c_grp_stride = 0; g.pos = nullptr; g.epi = epi;
    return g;
}

bool skinny_ok(const GemmArgs& g) {
    // very wide N (logits) at >= 24 rows: the 128x128 LDS-tiled kernel streams the
    // weights faster (measured 36 vs 44 us at M = 64, N = 51866)
    // (32-row skinny groups for the 64-row logits, which would fit beside another lane's
    // encoder workgroup: 4707 vs 4789 audio-s/s, measured; again with the fragment-major
    // weights in round 4: 5020 / 5019 vs 5065 / 5048, gpurun_out/r04_ag)
    if (g.N >= 16384 && g.M >= 24) return false;
    return g.M <= 64 && g.K % 128 == 0 &&
           (g.epi == EPI_F16 || g.epi == EPI_F16_GELU || g.epi == EPI_F32_RESID || g.epi == EPI_F32);
}

void run_gemm(osw_ctx* c, const GemmArgs& g0, int cls) {
    GemmArgs g = g0;
    g.share_cus = c->share_cus;
    REQUIRE(g.K % 64 == 0, "GEMM K must be a multiple of 64");
    REQUIRE(!g.A_lo || g.epi == EPI_F32, "hi/lo operands feed fp32 outputs only");
    const bool skinny = skinny_ok(g);
    // the tiled kernels' non-fp32 epilogues leave through an LDS image in 16-B chunks
    // (staged_epilogue_sq, the 256-tile staged epilogues) and check only each chunk's
    // first column against N: every row start must be 16-B aligned and N whole chunks
    REQUIRE(skinny || g.epi == EPI_F32 ||
                (g.N % 8 == 0 && (g.epi == EPI_HEADS || (g.ldc % 8 == 0 && g.c_grp_stride % 8 == 0))),
            "GEMM epilogue needs N, ldc and the C group stride to be multiples of 8");
    Timed t(c, cls, 2.0 * g.M * g.N * g.K);
    if (skinny) {
        REQUIRE((int64_t)skinny_ksplit(g.N, g.K) * g.M * g.N <= c->part_floats, "split-K workspace too small");
        launch_gemm_skinny(g, c->part, c->stream);
    } else {
        launch_gemm(g, c->stream);
    }
    HIPCHK(hipGetLastError());
}

// ---------------------------- encoder --------------------------------------
void encoder_layer(osw_ctx* c, int i, int nb) {
    const osw_dims& d = c->d;
    const int De = d.n_audio_state, H = d.n_audio_head;
    const int M = nb * T_ENC;
    const std::string p = "enc.l" + std::to_string(i);
    launch_layernorm(c->X, M, De, WF(c, p + ".ln1.g"), WF(c, p + ".ln1.b"), c->Xn, c->stream);
    GemmArgs g = gemm_plain(c->Xn, De, WH(c, p + ".qkv.w"), WF(c, p + ".qkv.b"), M, 3 * De, De, c->QKV, 0, EPI_HEADS);
    g.heads_T = T_ENC; g.heads_H = H; g.heads_nb = nb;
    run_gemm(c, g, CL_ENC_GEMM);
    {
        Timed t(c, CL_ENC_ATTN, 4.0 * nb * H * (double)T_ENC * T_ENC * 64);
        launch_enc_attn(c->QKV, c->O, T_ENC, H, nb, c->stream);
        HIPCHK(hipGetLastError());
    }
    run_gemm(c, gemm_plain(c->O, De, WH(c, p + ".o.w"), WF(c, p + ".o.b"), M, De, De, c->X, De, EPI_F32_RESID),
             CL_ENC_GEMM);
    launch_layernorm(c->X, M, De, WF(c, p + ".ln2.g"), WF(c, p + ".ln2.b"), c->Xn, c->stream);
    run_gemm(c, gemm_plain(c->Xn, De, WH(c, p + ".fc1.w"), WF(c, p + ".fc1.b"), M, 4 * De, De, c->Hf, 4 * De,
                           EPI_F16_GELU), CL_ENC_GEMM);
    run_gemm(c, gemm_plain(c->Hf, 4 * De, WH(c, p + ".fc2.w"), WF(c, p + ".fc2.b"), M, De, 4 * De, c->X, De,
                           EPI_F32_RESID), CL_ENC_GEMM);
}

// slots (row refill): window i's cross K/V goes to decoder row slots[i] of a c->B-row layout
void encode(osw_ctx* c, const osw_window* wins, int n, const int* slots = nullptr) {
    REQUIRE(c->finalized, "weights not finalized");
    REQUIRE(n >= 1 && n <= c->B, "window count out of range");
    const osw_dims& d = c->d;
    const int De = d.n_audio_state;
    if (slots) {
        std::vector<char> seen(c->B, 0);
        for (int i = 0; i < n; ++i) {
            REQUIRE(slots[i] >= 0 && slots[i] < c->B && !seen[slots[i]], "refill slots must be distinct rows < max_batch");
            seen[slots[i]] = 1;
        }
    }
    std::vector<int> hw(3 * n);
    for (int i = 0; i < n; ++i) {
        REQUIRE(wins[i].clip >= 0 && wins[i].clip < c->n_clips, "window clip out of range");
        REQUIRE(wins[i].seek >= 0 && wins[i].seek < c->nframes[wins[i].clip], "window seek out of range");
        REQUIRE(wins[i].segment_size >= 1, "empty window");
        hw[i] = wins[i].clip;
        hw[n + i] = wins[i].seek;
        hw[2 * n + i] = std::min(wins[i].segment_size, N_FR);
    }
    HIPCHK(hipMemcpyAsync(c->win, hw.data(), hw.size() * 4, hipMemcpyHostToDevice, c->stream));
    std::unique_lock<std::mutex> baton;  // held while this encoder is enqueued (EncBaton)
    // Encoders of fewer than c->baton_min (9) windows skip the baton: a streaming call's
    // 1-4-window encoder fills a fraction of the GPU, so sibling lanes' small encoders run
    // side by side.  Basis: the 4-concurrent-caller probe, 161.6 -> 169.0 calls/s
    // (gpurun_out/r03_ai); the config-5 simulation moved 149.0 -> 154.9 calls/s in that run,
    // but it spreads 148.6-156.0 run to run, so its gain is within noise.
    // The 64-window batches keep the baton.
    if (c->baton && n >= c->baton_min) baton = std::unique_lock<std::mutex>(c->baton->mu);
    // the encoder's kernels go to the low-priority encoder stream (swapped in as c->stream
    // for the launch helpers), fenced by events on both sides
    hipStream_t dec_stream = c->stream;
    struct Restore {
        osw_ctx* c;
        hipStream_t s;
        bool share;
        ~Restore() { c->stream = s; c->share_cus = share; }
    } restore{c, dec_stream, c->share_cus};
    // the CU reservation for sibling decoders (GemmArgs::share_cus) only for the batched
    // encoders: the small ones (streaming calls, session admissions) finish sooner on
    // every CU (OSW_GEMM_GRID=256 in the config-5 simulation: 158.6 -> 164.0 calls/s)
    static const bool share_small = getenv("OSW_SHARE_SMALL") != nullptr;  // A/B switch
    if (n < c->baton_min && !share_small) c->share_cus = false;
    if (c->enc_stream) {
        HIPCHK(hipEventRecord(c->enc_in, dec_stream));
        HIPCHK(hipStreamWaitEvent(c->enc_stream, c->enc_in, 0));
        c->stream = c->enc_stream;
    }
    if (baton.owns_lock() && c->baton->recorded) HIPCHK(hipStreamWaitEvent(c->stream, c->baton->ev, 0));
    {
        Timed t(c, CL_STAGE_ENC, 0);
        launch_mel_window(c->logmel, c->mel_off_d, c->nframes_d, c->clip_max, c->win, c->win + n, c->win + 2 * n, n,
                          d.n_mels, c->C1, c->X1, c->stream);
        // conv1: A row (w, t) = X1[w][t .. t+2][:] (3 rows of C1) ; C row -> H1[w][1 + t]
        GemmArgs g{};
        g.A = c->X1; g.lda = c->C1; g.a_grp_rows = N_FR; g.a_grp_stride = 3002LL * c->C1;
        g.W = WH(c, "enc.conv1.w"); g.ldw = 3 * c->C1; g.bias = WF(c, "enc.conv1.b");
        g.M = n * N_FR; g.N = De; g.K = 3 * c->C1;
        g.C = c->H1 + De; g.ldc = De; g.c_grp_rows = N_FR; g.c_grp_stride = 3001LL * De; g.epi = EPI_F16_GELU;
        run_gemm(c, g, CL_ENC_GEMM);
        // conv2 (stride 2): A row (w, t) = H1[w][2t .. 2t+2][:]  (H1 row r = input frame r-1)
        GemmArgs g2{};
        g2.A = c->H1; g2.lda = 2LL * De; g2.a_grp_rows = T_ENC; g2.a_grp_stride = 3001LL * De;
        g2.W = WH(c, "enc.conv2.w"); g2.ldw = 3LL * De; g2.bias = WF(c, "enc.conv2.b");
        g2.M = n * T_ENC; g2.N = De; g2.K = 3 * De;
        g2.C = c->X; g2.ldc = De; g2.c_grp_rows = T_ENC; g2.c_grp_stride = (int64_t)T_ENC * De;
        g2.pos = WF(c, "enc.pos"); g2.epi = EPI_F32_GELU_POS;
        run_gemm(c, g2, CL_ENC_GEMM);
        for (int i = 0; i < d.n_audio_layer; ++i) encoder_layer(c, i, n);
        launch_layernorm(c->X, (int64_t)n * T_ENC, De, WF(c, "enc.lnpost.g"), WF(c, "enc.lnpost.b"), c->E, c->stream);
    }
    {
        Timed t(c, CL_STAGE_XKV, 0);
        GemmArgs g = gemm_plain(c->E, De, WH(c, "dec.crosskv.w"), WF(c, "dec.crosskv.b"), n * T_ENC,
                                d.n_text_layer * 2 * d.n_text_state, De, c->XKV, 0, EPI_HEADS);
        g.heads_T = T_ENC; g.heads_H = d.n_text_head; g.heads_nb = n;
        if (slots) {
            HIPCHK(hipMemcpyAsync(c->slot_d, slots, (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
            g.heads_nb = c->B;
            g.heads_slot = c->slot_d;
        }
        run_gemm(c, g, 0);
    }
    HIPCHK(hipGetLastError());
    if (baton.owns_lock()) {
        HIPCHK(hipEventRecord(c->baton->ev, c->stream));
        c->baton->recorded = true;
    }
    if (c->enc_stream) {
        HIPCHK(hipEventRecord(c->enc_out, c->enc_stream));
        HIPCHK(hipStreamWaitEvent(dec_stream, c->enc_out, 0));
    }
    c->n_encoded = n;
}

// ---------------------------- decoder --------------------------------------
// One decoder row (batch-1 latency; PRO_ROWS): the
// residual+LayerNorm and GELU-reduce kernels are not launched; each runs as the prologue
// of the projection that consumes it (gemm_skinny_kernel<.., PRO>, resln.h), and the
// embedding is the prologue of layer 0's qkv: 51 -> 34 launches per step, 4 x [qkv,
// self-attn, o, q, cross-attn, xo, fc1, fc2] + logits + select.  The residual stream
// ping-pongs between xd and xd2 (every workgroup of a GEMM reads x, one writes x'), the
// slabs between part and part2 (a GEMM's prologue reads its producer's slabs while its
// epilogue writes its own).  Same arithmetic as decoder_step's separate kernels.
void decoder_step_fused(osw_ctx* c, int nb, int group, bool gather, const SelFuse* sf) {
    const osw_dims& d = c->d;
    const int D = d.n_text_state, H = d.n_text_head, L = d.n_text_layer, ctx = d.n_text_ctx;
    const int64_t xkv_which = (int64_t)(c->xkv_windows ? c->xkv_windows : nb / group) * H * T_ENC * 64;
    const int64_t kv_layer = (int64_t)(c->kv_rows ? c->kv_rows : nb) * H * ctx * 64;
    const int64_t lo_d = (int64_t)c->R * D;
    float* xs[2] = {c->xd, c->xd2};
    float* ps[2] = {c->part, c->part2};
    int xi = 0, last = 1, ks = 0;  // residual buffer holding x; slab buffer of the last GEMM
    auto gemm = [&](const h16* A, const std::string& w, int N, int K) {
        GemmArgs g = gemm_plain(A, D, WH(c, w), nullptr, nb, N, K, nullptr, 0, EPI_F32);
        g.Wf = WFR(c, w);
        g.A_lo = A ? A + lo_d : nullptr;
        return g;
    };
    // residual + LayerNorm prologue over the last GEMM's slabs (bias = its bias); part ==
    // nullptr: the embedding entry
    auto resln = [&](const float* bias, const std::string& ln, bool embed) {
        ProArgs pa{};
        pa.ln = ResLnArgs{embed ? nullptr : ps[last], ks, (int64_t)nb * D, bias, xs[xi], xs[xi ^ 1],
                          WF(c, ln + ".g"), WF(c, ln + ".b"), WH(c, "dec.tok"), WF(c, "dec.pos"), c->cur_tok, c->pos,
                          ctx, D, d.n_vocab, c->row_pos ? 1 : 0};
        xi ^= 1;
        return pa;
    };
    auto plain = [&](const h16* A, const std::string& w, int N, int K) {
        ks = launch_gemm_skinny_partial(gemm(A, w, N, K), ps[last ^ 1], c->stream);
        last ^= 1;
    };
    auto fused = [&](int pro, const ProArgs& pa, const std::string& w, int N, int K) {
        ks = launch_gemm_skinny_pro(gemm(nullptr, w, N, K), pro, pa, false, ps[last ^ 1], c->stream);
        last ^= 1;
    };
    // OSW_B1_ATTN_TAIL=1: the self-attention as the qkv GEMM's last-arriver tail per head
    // (TAIL_ATTN, the same device function as the standalone kernel, so the same bits; the
    // whole GPU suite is green with it).  Measured slower: the tailed qkv takes 15.9 us per
    // launch against 8.0 + 6.4 us for the GEMM and the self-attention kernel, batch-1 p50
    // 111.4 / 111.6 vs 107.1 / 108.7 ms (profiles/r06_s2d_b1_attn_tail_ab.txt): the in-launch
    // seam (ticket, device-scope slab loads) costs more than the kernel boundary it removes
    static const bool attn_tail_on = [] {
        const char* e = getenv("OSW_B1_ATTN_TAIL");
        return e && e[0] == '1';
    }();
    const bool attn_tail = attn_tail_on && nb == 1 && !gather;
    for (int l = 0; l < L; ++l) {
        const std::string p = "dec.l" + std::to_string(l), pp = "dec.l" + std::to_string(l - 1);
        ProArgs pq = l == 0 ? resln(nullptr, p + ".ln1", true) : resln(WF(c, pp + ".fc2.b"), p + ".ln1", false);
        if (attn_tail) {
            pq.tail_ticket = c->tail_ticket + 2048;  // [H] (the GELU tails use the first 160)
            pq.attn = SelfAttnTail{WF(c, p + ".qkv.b"), c->kc + l * kv_layer, c->vc + l * kv_layer, c->pos, H, ctx,
                                   c->row_pos ? 1 : 0, c->dattn, lo_d, c->sel};
            ks = launch_gemm_skinny_pro(gemm(nullptr, p + ".qkv.w", 3 * D, D), PRO_RESLN, pq, false, ps[last ^ 1],
                                        c->stream, false, true);
            last ^= 1;
        } else {
            fused(PRO_RESLN, pq, p + ".qkv.w", 3 * D, D);
            launch_dec_self_attn(ps[last], ks, WF(c, p + ".qkv.b"), c->kc + l * kv_layer, c->vc + l * kv_layer, c->pos,
                                 nb, H, ctx, c->dattn, lo_d, gather ? c->anc : nullptr, group, c->sel, c->stream,
                                 c->row_pos);
        }
        plain(c->dattn, p + ".o.w", D, D);
        fused(PRO_RESLN, resln(WF(c, p + ".o.b"), p + ".ln2", false), p + ".xq.w", D, D);
        {
            Timed t(c, CL_XATTN, 2.0 * nb * H * (double)T_ENC * 64 * 2);
            launch_dec_cross_attn(ps[last], ks, WF(c, p + ".xq.b"), c->XKV + (2 * l) * xkv_which,
                                  c->XKV + (2 * l + 1) * xkv_which, nb, H, T_ENC, group, c->dattn, lo_d, c->xws,
                                  c->xticket, c->sel, c->stream);
        }
        plain(c->dattn, p + ".xo.w", D, D);
        fused(PRO_RESLN, resln(WF(c, p + ".xo.b"), p + ".ln3", false), p + ".fc1.w", 4 * D, D);
        ProArgs pg{};
        pg.part = ps[last]; pg.ks = ks; pg.bias = WF(c, p + ".fc1.b");
        fused(PRO_GELU, pg, p + ".fc2.w", D, 4 * D);
    }
    const std::string pl = "dec.l" + std::to_string(L - 1);
    GemmArgs gl = gemm(nullptr, "dec.tok", d.n_vocab, D);
    gl.C = c->logits;
    gl.ldc = d.n_vocab;
    ProArgs pl_args = resln(WF(c, pl + ".fc2.b"), "dec.lnpost", false);
    if (sf) pl_args.sel = *sf;
    launch_gemm_skinny_pro(gl, PRO_RESLN, pl_args, true, nullptr, c->stream, sf != nullptr);
    HIPCHK(hipGetLastError());
}

// One decoder step for nb windows.  Every projection is a split-K skinny GEMM whose
// partial slabs are reduced by the kernel that consumes them (self/cross attention
// for q/k/v, residual+LayerNorm for the out-projections and fc2, GELU for fc1).
// nb = decoder rows (windows x group); the `group` rows of one window are adjacent
// (beam hypotheses or best_of samples); `gather` = beam rows read the self-K/V cache
// through the ancestry table.
// sf (batch-1 greedy): the logits GEMM also selects the token and advances the step
// counter; returns whether it did (the caller then launches no select).
bool decoder_step(osw_ctx* c, int nb, int group, bool gather, const SelFuse* sf = nullptr) {
    const osw_dims& d = c->d;
    const int D = d.n_text_state, H = d.n_text_head, L = d.n_text_layer, ctx = d.n_text_ctx;
    const int64_t xkv_which = (int64_t)(c->xkv_windows ? c->xkv_windows : nb / group) * H * T_ENC * 64;
    const int64_t kv_layer = (int64_t)(c->kv_rows ? c->kv_rows : nb) * H * ctx * 64;
    REQUIRE(nb <= c->R && D <= 1280, "decoder step: rows <= capacity and D <= 1280");
    REQUIRE(ctx <= 448, "decoder self-attention holds at most 448 positions");
    // the decoder's GEMM operands are hi/lo fp16 pairs (fp32-accurate activations: the
    // logits stay within 1e-3 of an fp32 decoder); lo = hi + R rows
    const int64_t lo_d = (int64_t)c->R * D, lo_4d = (int64_t)c->R * 4 * D;
    // <= 64 rows: split-K skinny GEMM; more (beam search): see below
    auto partial = [&](const h16* A, int lda, const std::string& w, int N, int K) {
        const h16* Wt = WH(c, w);
        const int64_t lo = lda == 4 * D ? lo_4d : lo_d;
        // > 64 rows (beam search): skinny row groups for every projection.  Round 3 put N > 1536
        // (qkv, fc1) on 64x128 split-K tiles (alone at 320 rows: N = 3840 12.8 vs 17.9 us,
        // N = 5120 20.4 vs 21.7); round 6 re-measured the whole beam-5 bench on one box: 3-lane
        // 3145 / 3138 (skinny everywhere) vs 3098 / 3104 audio-s/s (tiles for N > 1536), one
        // lane 2617 / 2613 vs 2647 / 2650 (profiles/r06_s2k_beam_gemm_ab.txt): the 16-KiB skinny
        // workgroups share the CUs with the other lanes' encoders better.  Same split-K depth
        // (kc 256) and MFMA order either way: the same bits.  OSW_BEAM_GEMM=1: the tiles for
        // N > 1536 (the round-3 choice), 3: tiles everywhere.
        static const int force = getenv("OSW_BEAM_GEMM") ? atoi(getenv("OSW_BEAM_GEMM")) : 2;
        if (nb > 64 && (force == 3 || (force == 1 && N > 1536))) {
            const int ks = tiled_ksplit(nb, N, K);
            REQUIRE((int64_t)ks * nb * N <= c->part_floats, "decoder workspace too small");
            GemmArgs g = gemm_plain(A, lda, Wt, nullptr, nb, N, K, nullptr, 0, EPI_F32);
            g.A_lo = A + lo;
            launch_gemm_tiled_partial(g, c->part, ks, c->stream);
            return ks;
        }
        GemmArgs g = gemm_plain(A, lda, Wt, nullptr, nb, N, K, nullptr, 0, EPI_F32);
        g.Wf = WFR(c, w);
        g.A_lo = A + lo;
        REQUIRE((int64_t)skinny_ksplit(N, K) * nb * N <= c->part_floats, "split-K workspace too small");
        return launch_gemm_skinny_partial(g, c->part, c->stream);
    };
    static const bool no_fuse = getenv("OSW_NO_FUSE") != nullptr;  // A/B switch
    if (nb <= PRO_ROWS && !no_fuse) {
        decoder_step_fused(c, nb, group, gather, nb == 1 ? sf : nullptr);
        return sf != nullptr && nb == 1;
    }
    static const bool no_gelu_pro = getenv("OSW_NO_GELU_PRO") != nullptr;  // A/B switch
    const bool gelu_pro = nb <= GELU_ROWS && !no_gelu_pro && 4 * D / skinny_ksplit(D, 4 * D) <= GELU_KC;
    // OSW_GELU_TAIL=1: fc1's last workgroup per column block reduces + GELUs its slabs (no
    // reduce kernel).  Measured slower in the 3-lane headline (5018 / 5016 vs 5049 audio-s/s,
    // profiles/r06_b_gelu_tail_ab.txt): with the lanes overlapping, a launch fewer buys less
    // than the serial tail costs, so it is opt-in
    static const bool gelu_tail_on = getenv("OSW_GELU_TAIL") && getenv("OSW_GELU_TAIL")[0] == '1';
    const bool gelu_tail = !gelu_pro && nb <= 64 && gelu_tail_on && (4 * D) % 64 == 0;
    // x = tok_emb[tok] + pos_emb[pos]; xdn = LN1_0(x)
    launch_dec_resid_ln(nullptr, 0, nb, D, nullptr, c->xd, WF(c, "dec.l0.ln1.g"), WF(c, "dec.l0.ln1.b"), c->xdn, lo_d,
                        WH(c, "dec.tok"), WF(c, "dec.pos"), c->cur_tok, c->pos, ctx, d.n_vocab, c->stream, c->row_pos);
    for (int l = 0; l < L; ++l) {
        const std::string p = "dec.l" + std::to_string(l);
        int ks = partial(c->xdn, D, p + ".qkv.w", 3 * D, D);
        launch_dec_self_attn(c->part, ks, WF(c, p + ".qkv.b"), c->kc + l * kv_layer, c->vc + l * kv_layer, c->pos, nb,
                             H, ctx, c->dattn, lo_d, gather ? c->anc : nullptr, group, c->sel, c->stream, c->row_pos);
        ks = partial(c->dattn, D, p + ".o.w", D, D);
        launch_dec_resid_ln(c->part, ks, nb, D, WF(c, p + ".o.b"), c->xd, WF(c, p + ".ln2.g"), WF(c, p + ".ln2.b"),
                            c->xdn, lo_d, nullptr, nullptr, nullptr, nullptr, ctx, d.n_vocab, c->stream);
        ks = partial(c->xdn, D, p + ".xq.w", D, D);
        {
            Timed t(c, CL_XATTN, 2.0 * nb * H * (double)T_ENC * 64 * 2);
            launch_dec_cross_attn(c->part, ks, WF(c, p + ".xq.b"), c->XKV + (2 * l) * xkv_which,
                                  c->XKV + (2 * l + 1) * xkv_which, nb, H, T_ENC, group, c->dattn, lo_d, c->xws,
                                  c->xticket, c->sel, c->stream);
        }
        ks = partial(c->dattn, D, p + ".xo.w", D, D);
        launch_dec_resid_ln(c->part, ks, nb, D, WF(c, p + ".xo.b"), c->xd, WF(c, p + ".ln3.g"), WF(c, p + ".ln3.b"),
                            c->xdn, lo_d, nullptr, nullptr, nullptr, nullptr, ctx, d.n_vocab, c->stream);
        // (a whole-K fc1 with the GELU epilogue fused has only N/64 = 80 workgroups at
        // turbo: 22.7 us vs 9.6 + 4.7 us for split-K + reduce, measured)
        const float* fc2_part = c->part;
        if (gelu_tail) {
            // 9..64 rows: split-K fc1 whose last workgroup per column block reduces that
            // block's slabs + bias + GELU (TAIL_GELU): no reduce kernel
            GemmArgs g = gemm_plain(c->xdn, D, WH(c, p + ".fc1.w"), nullptr, nb, 4 * D, D, nullptr, 0, EPI_F32);
            g.Wf = WFR(c, p + ".fc1.w");
            g.A_lo = c->xdn + lo_d;
            ProArgs pt{};
            pt.bias = WF(c, p + ".fc1.b");
            pt.tail_ticket = c->tail_ticket;
            pt.tail_y = c->dh;
            pt.tail_lo = lo_4d;
            launch_gemm_skinny_gelu_tail(g, c->part, pt, c->stream);
            HIPCHK(hipGetLastError());
            ks = partial(c->dh, 4 * D, p + ".fc2.w", D, 4 * D);
        } else {
        ks = partial(c->xdn, D, p + ".fc1.w", 4 * D, D);
        if (gelu_pro) {
            // <= 8 rows: the GELU reduce is fc2's prologue (each workgroup reduces only its own
            // K range of the fc1 slabs, resln.h), fc2's slabs go to part2
            ProArgs pg{};
            pg.part = c->part; pg.ks = ks; pg.bias = WF(c, p + ".fc1.b");
            GemmArgs g = gemm_plain(nullptr, D, WH(c, p + ".fc2.w"), nullptr, nb, D, 4 * D, nullptr, 0, EPI_F32);
            g.Wf = WFR(c, p + ".fc2.w");
            ks = launch_gemm_skinny_pro(g, PRO_GELU, pg, false, c->part2, c->stream);
            fc2_part = c->part2;
        } else {
            launch_dec_reduce_gelu(c->part, ks, nb, 4 * D, WF(c, p + ".fc1.b"), c->dh, lo_4d, c->stream);
            ks = partial(c->dh, 4 * D, p + ".fc2.w", D, 4 * D);
        }
        }
        const std::string nx = l + 1 < L ? "dec.l" + std::to_string(l + 1) + ".ln1" : std::string("dec.lnpost");
        launch_dec_resid_ln(fc2_part, ks, nb, D, WF(c, p + ".fc2.b"), c->xd, WF(c, nx + ".g"), WF(c, nx + ".b"), c->xdn,
                            lo_d, nullptr, nullptr, nullptr, nullptr, ctx, d.n_vocab, c->stream);
    }
    GemmArgs gl = gemm_plain(c->xdn, D, WH(c, "dec.tok"), nullptr, nb, d.n_vocab, D, c->logits, d.n_vocab, EPI_F32);
    gl.Wf = WFR(c, "dec.tok");  // used by the skinny kernel (< 24 rows); the wide kernel reads W
    gl.A_lo = c->xdn + lo_d;
    run_gemm(c, gl, 0);
    return false;
}

// The decode graph for `key` (CH steps of one_step), captured and instantiated on first use;
// at most 16 per context, the least recently used one destroyed to make room.
hipGraphExec_t decode_graph(osw_ctx* c, const std::vector<int64_t>& key, const std::function<void()>& one_step,
                            int CH) {
    auto hit = c->dgraphs.find(key);
    if (hit != c->dgraphs.end()) {
        hit->second.second = ++c->dgraph_tick;
        return hit->second.first;
    }
    {
        constexpr size_t kMaxGraphs = 16;
        // A sibling lane's encoder waits on the baton event, which this lane may have
        // recorded on this stream: HIP refuses that wait while this stream captures
        // ("dependency created on uncaptured work in another stream"), so no sibling
        // enqueues an encoder (which holds the baton's mutex) during a capture.  And no
        // thread of the process touches the legacy stream or synchronises implicitly while
        // it captures: the capture gate (capture_gate) is held from here to the instantiation.
        std::unique_lock<std::mutex> no_encoder;
        if (c->baton) no_encoder = std::unique_lock<std::mutex>(c->baton->mu);
        GateLock gate_(capture_gate());
        if (c->dgraphs.size() >= kMaxGraphs) {  // evict the least recently used
            auto lru = c->dgraphs.begin();
            for (auto it = c->dgraphs.begin(); it != c->dgraphs.end(); ++it)
                if (it->second.second < lru->second.second) lru = it;
            HIPCHK(hipStreamSynchronize(c->stream));
            trace_graph(c, "destroy (LRU)");
            HIPCHK(hipGraphExecDestroy(lru->second.first));
            c->dgraphs.erase(lru);
        }
        HIPCHK(hipStreamSynchronize(c->stream));
        hipGraph_t gr = nullptr;
        hipGraphExec_t ge = nullptr;
        c->capturing = true;
        try {
            trace_graph(c, "capture begin");
            HIPCHK(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
            for (int i = 0; i < CH; ++i) one_step();
            HIPCHK(hipStreamEndCapture(c->stream, &gr));
            trace_graph(c, "capture end");
        } catch (...) {
            c->capturing = false;
            hipGraph_t junk = nullptr;
            (void)hipStreamEndCapture(c->stream, &junk);
            if (junk) (void)hipGraphDestroy(junk);
            throw;
        }
        c->capturing = false;
        hipError_t e = hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
        trace_graph(c, "instantiated");
        (void)hipGraphDestroy(gr);
        HIPCHK(e);
        c->dgraphs[key] = {ge, ++c->dgraph_tick};
        return ge;
    }
}

void decode(osw_ctx* c, int nb, const osw_decode_opts* o, osw_window_result* r) {
    REQUIRE(nb >= 1 && nb == c->n_encoded, "decode window count must equal the last encode call");
    REQUIRE(o && r && r->tokens && r->n_tokens && r->sum_logprob && r->no_speech_prob && r->language,
            "null decode argument");
    const osw_dims& d = c->d;
    const int V = d.n_vocab;
    const int n_pre = o->n_prefix;
    REQUIRE(n_pre >= 0 && (n_pre == 0 || o->prefix_tokens), "bad prefix");
    // temperature > 0 (faster-whisper's sampling branch): beam 1 and best_of independent
    // sampled rows per window, the best one kept; otherwise beam search or greedy
    const bool sampling = o->temperature > 0.f;
    const int beam = sampling ? 1 : std::max(1, o->beam_size);
    const int group = sampling ? std::max(1, o->best_of) : beam;  // decoder rows per window
    REQUIRE(group <= MAX_BEAM, "beam_size / best_of > 8");
    const int rows = nb * group;
    REQUIRE(rows <= c->R, "windows x beam_size (best_of) exceeds the decoder row capacity (5 x max_batch)");
    REQUIRE(group == 1 || !r->logits_dump, "logits dump needs one decoder row per window");
    REQUIRE(V <= SEL_SPLIT * 4096, "vocabulary too large for the selection kernels");
    const int P = n_pre + 3 + (o->without_timestamps ? 1 : 0);
    const int max_len = std::min(o->max_length > 0 ? o->max_length : d.n_text_ctx, d.n_text_ctx);
    REQUIRE(P < max_len, "prompt longer than max_length");
    // one prompt per decoder row (the beam rows of a window share it)
    std::vector<int> prompt((size_t)rows * P);
    for (int b = 0; b < nb; ++b)
        for (int k = 0; k < group; ++k) {
            int* pr = &prompt[((size_t)b * group + k) * P];
            for (int i = 0; i < n_pre; ++i) pr[i] = o->prefix_tokens[(size_t)b * n_pre + i];
            pr[n_pre] = o->sot;
            pr[n_pre + 1] = o->language_tokens ? o->language_tokens[b] : o->language_token;  // -1: detect
            pr[n_pre + 2] = o->task_token;
            if (o->without_timestamps) pr[n_pre + 3] = o->no_timestamps;
        }
    std::vector<unsigned> mask((V + 31) / 32, 0u);
    for (int i = 0; i < o->n_suppress; ++i) {
        const int t = o->suppress_tokens[i];
        if (t >= 0 && t < V) mask[t >> 5] |= 1u << (t & 31);
    }
    std::vector<int> first(rows);
    for (int b = 0; b < rows; ++b) first[b] = prompt[(size_t)b * P];
    HIPCHK(hipMemcpyAsync(c->prompt, prompt.data(), prompt.size() * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->supmask, mask.data(), mask.size() * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->cur_tok, first.data(), rows * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemsetAsync(c->pos, 0, 4, c->stream));
    HIPCHK(hipMemsetAsync(c->sel, 0, (size_t)rows * sizeof(SelState), c->stream));
    const int max_tok = std::max(1, max_len - P);
    std::vector<int> anc0;
    if (beam > 1) {
        anc0.resize((size_t)rows * d.n_text_ctx);
        for (int b = 0; b < rows; ++b)
            for (int p = 0; p < d.n_text_ctx; ++p) anc0[(size_t)b * d.n_text_ctx + p] = b;
        HIPCHK(hipMemcpyAsync(c->anc, anc0.data(), anc0.size() * 4, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemsetAsync(c->bwin, 0, (size_t)nb * sizeof(BeamWin), c->stream));
        HIPCHK(hipMemsetAsync(c->btok, 0, (size_t)nb * max_tok * 4, c->stream));
    }
    SelParams SP{};
    SP.prompt_len = P; SP.sot_pos = n_pre; SP.lang_pos = n_pre + 1; SP.max_length = max_len;
    SP.pstride = P; SP.tail = P - n_pre;
    SP.V = V; SP.eot = o->eot; SP.no_speech = o->no_speech; SP.no_ts = o->no_timestamps; SP.tb = o->timestamp_begin;
    SP.blank = o->blank; SP.first_lang = o->first_lang; SP.n_langs = o->n_langs;
    SP.suppress_blank = o->suppress_blank; SP.with_ts = o->without_timestamps ? 0 : 1;
    SP.max_init_ts = o->max_initial_timestamp_index;
    SP.beam = beam;
    SP.num_hyp = std::max(1, o->num_hypotheses);
    SP.max_cand = std::max(1, (int)std::lround(beam * (o->patience > 0.f ? o->patience : 1.f)));
    SP.length_penalty = o->length_penalty;
    SP.inv_temp = sampling ? 1.f / o->temperature : 0.f;
    HIPCHK(hipMemcpyAsync(c->seed_d, &o->seed, 8, hipMemcpyHostToDevice, c->stream));
    SP.seed = c->seed_d;
    SP.budget = nullptr;
    if (o->token_budget) {
        std::vector<int> bud(rows);
        for (int i = 0; i < rows; ++i) bud[i] = o->token_budget[i / group];
        HIPCHK(hipMemcpyAsync(c->budget, bud.data(), rows * 4, hipMemcpyHostToDevice, c->stream));
        SP.budget = c->budget;
    }
    auto select = [&] {
        launch_select(c->logits, rows, c->pos, SP, c->prompt, c->supmask, c->sel, c->cur_tok, c->tokens, max_tok,
                      c->selp, c->sel_arrive, beam == 1, c->bcand, c->stream);
        if (beam > 1)
            launch_beam(c->logits, nb, c->pos, SP, c->supmask, c->sel, c->selp, c->bcand, c->tokens, c->anc,
                        d.n_text_ctx, c->bwin, c->btok, c->cur_tok, max_tok, c->sel_arrive, c->stream);
    };
    // batch-1 greedy: the selection runs in the logits GEMM's epilogue (SelFuse, decode.h)
    static const bool no_fuse_sel = getenv("OSW_NO_FUSE_SELECT") != nullptr;  // A/B switch
    SelFuse sf{SP, c->logits, c->pos, c->supmask, c->prompt, c->sel, c->cur_tok, c->tokens, max_tok, c->selp1,
               c->sel_arrive + 1};
    const SelFuse* sfp = (rows == 1 && beam == 1 && !sampling && !no_fuse_sel) ? &sf : nullptr;
    auto one_step = [&] {
        // the select kernel (greedy), the beam update or the fused selection advances the step counter
        if (!decoder_step(c, rows, group, beam > 1, sfp)) select();
    };
    const int CH = 8;
    const bool graph = c->use_graph && !r->logits_dump && !c->prof_eager;
    if (graph) {
        int32_t lp_bits, it_bits;
        std::memcpy(&lp_bits, &SP.length_penalty, 4);
        std::memcpy(&it_bits, &SP.inv_temp, 4);
        std::vector<int64_t> key = {nb, P, n_pre, max_len, o->eot, o->no_speech, o->no_timestamps,
                                    o->timestamp_begin, o->blank, o->first_lang, o->n_langs, o->suppress_blank,
                                    o->without_timestamps, o->max_initial_timestamp_index, beam, SP.num_hyp,
                                    SP.max_cand, lp_bits, group, it_bits, SP.budget ? 1 : 0};
        c->dgraph = decode_graph(c, key, one_step, CH);
    }
    int steps = 0;
    {
        Timed t(c, CL_STAGE_DEC, 0);
        int since_check = 0;
        while (steps < max_len) {
            int did;
            if (graph && max_len - steps >= CH) {
                trace_graph(c, "launch");
                HIPCHK(hipGraphLaunch(c->dgraph, c->stream));
                did = CH;
            } else {
                const int samp = steps - (P - 1);
                if (r->logits_dump && samp >= 0 && samp < r->dump_steps) {
                    const bool selected = decoder_step(c, rows, group, beam > 1, sfp);
                    for (int b = 0; b < nb; ++b)
                        HIPCHK(hipMemcpyAsync(r->logits_dump + ((size_t)b * r->dump_steps + samp) * V,
                                              c->logits + (size_t)b * V, (size_t)V * 4, hipMemcpyDeviceToHost,
                                              c->stream));
                    if (!selected) select();
                } else {
                    one_step();
                }
                did = 1;
            }
            HIPCHK(hipGetLastError());
            steps += did;
            since_check += did;
            if (steps >= P && (since_check >= CH || steps >= max_len)) {
                since_check = 0;
                launch_count_done(c->sel, rows, c->done, c->stream);
                HIPCHK(hipMemcpyAsync(c->done_host, c->done, 4, hipMemcpyDeviceToHost, c->stream));
                HIPCHK(hipStreamSynchronize(c->stream));
                if (*c->done_host >= rows) break;
            }
        }
    }
    c->pf.decode_steps = steps;
    // read back
    std::vector<SelState> st(rows);
    HIPCHK(hipMemcpyAsync(st.data(), c->sel, rows * sizeof(SelState), hipMemcpyDeviceToHost, c->stream));
    std::vector<int> toks((size_t)(beam > 1 ? nb : rows) * max_tok);
    std::vector<BeamWin> bw(nb);
    if (beam > 1) {
        HIPCHK(hipMemcpyAsync(toks.data(), c->btok, toks.size() * 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(bw.data(), c->bwin, nb * sizeof(BeamWin), hipMemcpyDeviceToHost, c->stream));
    } else {
        HIPCHK(hipMemcpyAsync(toks.data(), c->tokens, toks.size() * 4, hipMemcpyDeviceToHost, c->stream));
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    // best_of: the sample with the highest sum_logprob / n**length_penalty (first on ties)
    auto norm = [&](const SelState& q) {
        if (q.n_sampled == 0) return o->length_penalty != 0.f ? -INFINITY : q.sum_lp;
        return q.sum_lp / std::pow((float)q.n_sampled, o->length_penalty);
    };
    for (int b = 0; b < nb; ++b) {
        size_t best = (size_t)b * group;
        if (sampling)
            for (int k = 1; k < group; ++k)
                if (norm(st[(size_t)b * group + k]) > norm(st[best])) best = (size_t)b * group + k;
        const SelState& sp = st[best];
        const int n0 = beam > 1 ? bw[b].best_len : sp.n_sampled;
        const int n = std::min(n0, std::min(max_tok, r->max_tokens));
        r->n_tokens[b] = n;
        const int* src = &toks[(beam > 1 ? (size_t)b : best) * max_tok];
        for (int i = 0; i < n; ++i) r->tokens[(size_t)b * r->max_tokens + i] = src[i];
        r->sum_logprob[b] = beam > 1 ? bw[b].best_raw : sp.sum_lp;
        r->no_speech_prob[b] = sp.nsp;
        r->language[b] = sp.lang;
    }
}

// Greedy decoding with row refill (osw_transcribe_refill): the decoder keeps c->B rows and
// every row has its own step counter (pos[row], SelParams::pos_row), so when a window
// finishes, a queued clip's window is encoded straight into that row's cross-K/V slot and
// starts at position 0 beside rows that are mid-way.  A batch then costs what its windows'
// own lengths cost instead of its longest window's.  Every row's arithmetic is the plain
// greedy decode's (rows are independent in every kernel), so each clip's result equals
// osw_transcribe_batch's for it.  Windows are admitted once refill_min rows are free (or
// when no row is active); empty rows stay finished and are skipped by the attention kernels.
void decode_refill(osw_ctx* c, int n_clips, const osw_decode_opts* o, osw_window_result* r, int refill_min) {
    REQUIRE(o && r && r->tokens && r->n_tokens && r->sum_logprob && r->no_speech_prob && r->language,
            "null decode argument");
    REQUIRE(!(o->temperature > 0.f) && o->beam_size <= 1, "row refill decodes greedily (temperature 0, beam_size 1)");
    REQUIRE(o->n_prefix == 0, "row refill takes no prefix tokens");
    REQUIRE(!r->logits_dump, "row refill has no logits dump");
    const osw_dims& d = c->d;
    const int V = d.n_vocab;
    REQUIRE(V <= SEL_SPLIT * 4096, "vocabulary too large for the selection kernels");
    const int R = c->B;
    REQUIRE(R <= c->R, "decoder rows");
    const int P = 3 + (o->without_timestamps ? 1 : 0);
    const int max_len = std::min(o->max_length > 0 ? o->max_length : d.n_text_ctx, d.n_text_ctx);
    REQUIRE(P < max_len, "prompt longer than max_length");
    const int max_tok = std::max(1, max_len - P);
    refill_min = std::max(1, std::min(refill_min, R));
    std::vector<unsigned> mask((V + 31) / 32, 0u);
    for (int i = 0; i < o->n_suppress; ++i) {
        const int t = o->suppress_tokens[i];
        if (t >= 0 && t < V) mask[t >> 5] |= 1u << (t & 31);
    }
    SelParams SP{};
    SP.prompt_len = P; SP.sot_pos = 0; SP.lang_pos = 1; SP.max_length = max_len;
    SP.pstride = P; SP.tail = P;
    SP.V = V; SP.eot = o->eot; SP.no_speech = o->no_speech; SP.no_ts = o->no_timestamps; SP.tb = o->timestamp_begin;
    SP.blank = o->blank; SP.first_lang = o->first_lang; SP.n_langs = o->n_langs;
    SP.suppress_blank = o->suppress_blank; SP.with_ts = o->without_timestamps ? 0 : 1;
    SP.max_init_ts = o->max_initial_timestamp_index;
    SP.beam = 1; SP.num_hyp = 1; SP.max_cand = 1;
    SP.length_penalty = o->length_penalty;
    SP.inv_temp = 0.f;
    HIPCHK(hipMemcpyAsync(c->seed_d, &o->seed, 8, hipMemcpyHostToDevice, c->stream));
    SP.seed = c->seed_d;
    SP.budget = o->token_budget ? c->budget : nullptr;
    SP.pos_row = 1;
    HIPCHK(hipMemcpyAsync(c->supmask, mask.data(), mask.size() * 4, hipMemcpyHostToDevice, c->stream));
    // every row starts finished (nothing to step until a window is admitted)
    std::vector<SelState> st(R);
    for (auto& q : st) q = SelState{}, q.done = 1;
    HIPCHK(hipMemcpyAsync(c->sel, st.data(), (size_t)R * sizeof(SelState), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemsetAsync(c->pos, 0, (size_t)R * 4, c->stream));
    HIPCHK(hipMemsetAsync(c->cur_tok, 0, (size_t)R * 4, c->stream));
    HIPCHK(hipMemsetAsync(c->prompt, 0, (size_t)R * P * 4, c->stream));
    struct RowPos {
        osw_ctx* c;
        ~RowPos() { c->row_pos = false; c->n_encoded = 0; }
    } row_pos_scope{c};
    c->row_pos = true;
    auto one_step = [&] {
        decoder_step(c, R, 1, false, nullptr);
        launch_select(c->logits, R, c->pos, SP, c->prompt, c->supmask, c->sel, c->cur_tok, c->tokens, max_tok,
                      c->selp, c->sel_arrive, true, c->bcand, c->stream);
    };
    const int CH = 8;
    const bool graph = c->use_graph && !c->prof_eager;
    hipGraphExec_t ge = nullptr;
    if (graph) {
        int32_t lp_bits;
        std::memcpy(&lp_bits, &SP.length_penalty, 4);
        // (the -1 tail keeps refill keys apart from decode()'s)
        const std::vector<int64_t> key = {R, P, 0, max_len, o->eot, o->no_speech, o->no_timestamps,
                                          o->timestamp_begin, o->blank, o->first_lang, o->n_langs, o->suppress_blank,
                                          o->without_timestamps, o->max_initial_timestamp_index, 1, 1,
                                          1, lp_bits, 1, 0, SP.budget ? 1 : 0, -1};
        ge = decode_graph(c, key, one_step, CH);
    }
    std::vector<int> row_clip(R, -1), pack, toks((size_t)R * max_tok);
    int next = 0, active = 0, steps = 0;
    while (true) {
        std::vector<int> free_rows;
        for (int i = 0; i < R; ++i)
            if (row_clip[i] < 0) free_rows.push_back(i);
        const int left = n_clips - next;
        if (left > 0 && (active == 0 || (int)free_rows.size() >= std::min(refill_min, left))) {
            const int k = std::min((int)free_rows.size(), left);
            std::vector<osw_window> wins(k);
            std::vector<int> slots(k);
            pack.assign((size_t)k * (2 + P), 0);
            for (int i = 0; i < k; ++i) {
                const int clip = next + i, row = free_rows[i];
                wins[i] = osw_window{clip, 0, std::max(1, std::min(N_FR, c->nframes[clip] - 1))};
                slots[i] = row;
                int* e = &pack[(size_t)i * (2 + P)];
                e[0] = row;
                e[1] = o->token_budget ? o->token_budget[clip] : 0;
                e[2] = o->sot;
                e[3] = o->language_tokens ? o->language_tokens[clip] : o->language_token;  // -1: detect
                e[4] = o->task_token;
                if (o->without_timestamps) e[5] = o->no_timestamps;
                row_clip[row] = clip;
            }
            encode(c, wins.data(), k, slots.data());
            c->n_encoded = 0;
            HIPCHK(hipMemcpyAsync(c->refill_pack, pack.data(), pack.size() * 4, hipMemcpyHostToDevice, c->stream));
            launch_refill_rows(c->refill_pack, k, P, c->prompt, SP.budget ? c->budget : nullptr, c->cur_tok, c->pos,
                               c->sel, c->stream);
            HIPCHK(hipGetLastError());
            next += k;
            active += k;
        }
        if (active == 0) break;
        if (graph) {
            trace_graph(c, "launch");
            HIPCHK(hipGraphLaunch(ge, c->stream));
        } else {
            for (int i = 0; i < CH; ++i) one_step();
        }
        HIPCHK(hipGetLastError());
        steps += CH;
        HIPCHK(hipMemcpyAsync(st.data(), c->sel, (size_t)R * sizeof(SelState), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        bool fin = false;
        for (int i = 0; i < R; ++i) fin |= row_clip[i] >= 0 && st[i].done;
        if (!fin) continue;
        HIPCHK(hipMemcpyAsync(toks.data(), c->tokens, toks.size() * 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        for (int i = 0; i < R; ++i) {
            const int clip = row_clip[i];
            if (clip < 0 || !st[i].done) continue;
            const SelState& q = st[i];
            const int n = std::min(q.n_sampled, std::min(max_tok, r->max_tokens));
            r->n_tokens[clip] = n;
            for (int j = 0; j < n; ++j) r->tokens[(size_t)clip * r->max_tokens + j] = toks[(size_t)i * max_tok + j];
            r->sum_logprob[clip] = q.sum_lp;
            r->no_speech_prob[clip] = q.nsp;
            r->language[clip] = q.lang;
            row_clip[i] = -1;
            --active;
        }
    }
    c->pf.decode_steps = steps;
}

// ------------------------------ mel ----------------------------------------
void log_mel(osw_ctx* c, const int16_t* pcm, const int64_t* offsets, int n, int on_device, int* nf_out) {
    REQUIRE(n >= 1, "need at least one clip");
    REQUIRE(pcm && offsets, "null pcm/offsets");
    const int n_mels = c->d.n_mels;
    const int64_t total = offsets[n] - offsets[0];
    REQUIRE(total >= 0, "bad offsets");
    std::vector<int64_t> offs(n + 1);
    for (int i = 0; i <= n; ++i) {
        offs[i] = offsets[i] - offsets[0];
        if (i) REQUIRE(offs[i] >= offs[i - 1], "offsets must be non-decreasing");
    }
    if (n > c->clips_cap) {
        const int cap = std::max(n, 2 * c->clips_cap);
        // superseded buffers are freed (hipFree waits for the device), not kept until destroy
        dfree(c->offsets, c->owned);
        dfree(c->mel_off_d, c->owned);
        dfree(c->nframes_d, c->owned);
        dfree(c->clip_max, c->owned);
        c->offsets = dalloc<int64_t>(cap + 1, c->owned);
        c->mel_off_d = dalloc<int64_t>(cap + 1, c->owned);
        c->nframes_d = dalloc<int>(cap, c->owned);
        c->clip_max = dalloc<int>(cap, c->owned);
        c->clips_cap = cap;
    }
    c->nframes.assign(n, 0);
    c->mel_off.assign(n + 1, 0);
    int max_nf = 0;
    for (int i = 0; i < n; ++i) {
        const int64_t N = offs[i + 1] - offs[i];
        c->nframes[i] = (int)((N + 160) / 160);
        c->mel_off[i + 1] = c->mel_off[i] + (int64_t)c->nframes[i] * n_mels;
        max_nf = std::max(max_nf, c->nframes[i]);
    }
    if ((size_t)c->mel_off[n] > c->logmel_cap) {
        c->logmel_cap = (size_t)c->mel_off[n] + (size_t)c->mel_off[n] / 2;
        dfree(c->logmel, c->owned);
        c->logmel = dalloc<float>(c->logmel_cap, c->owned);
    }
    const int16_t* src = pcm + offsets[0];
    if (!on_device) {
        if ((size_t)total > c->pcm_cap) {
            c->pcm_cap = (size_t)total + (size_t)total / 2 + 1;
            dfree(c->pcm, c->owned);
            c->pcm = dalloc<int16_t>(c->pcm_cap, c->owned);
        }
        if (total) HIPCHK(hipMemcpyAsync(c->pcm, src, (size_t)total * 2, hipMemcpyHostToDevice, c->stream));
        src = c->pcm;
    }
    HIPCHK(hipMemcpyAsync(c->offsets, offs.data(), (n + 1) * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->mel_off_d, c->mel_off.data(), (n + 1) * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->nframes_d, c->nframes.data(), n * 4, hipMemcpyHostToDevice, c->stream));
    {
        Timed t(c, CL_STAGE_MEL, 0);
        Timed k(c, CL_MEL, (double)total * 2 + (double)c->mel_off[n] * 4);
        launch_mel(src, c->offsets, c->mel_off_d, c->nframes_d, n, max_nf, c->tw400, c->hann, c->flo, c->fcnt,
                   c->foff, c->fw, n_mels, c->logmel, c->clip_max, c->stream);
        HIPCHK(hipGetLastError());
    }
    c->n_clips = n;
    if (nf_out)
        for (int i = 0; i < n; ++i) nf_out[i] = c->nframes[i];
}

// ------------------------------ ingest --------------------------------------
// Per-device state of the context-free ingest entry points (osw_ingest_*): a stream
// and scratch buffers grown on demand, one mutex per device.
struct IngestDev {
    std::mutex mu;
    hipStream_t s = nullptr;
    std::vector<void*> owned;
    int16_t* in = nullptr;
    size_t in_cap = 0;
    int16_t* out = nullptr;
    size_t out_cap = 0;
    float* sums = nullptr;   // [full blocks | tail leaves]
    size_t sums_cap = 0;
    int2* leaves = nullptr;  // tail leaves (<= 128)
    float* taps = nullptr;
    size_t taps_cap = 0;
};
std::mutex g_ingest_mu;
std::map<int, std::unique_ptr<IngestDev>> g_ingest;

IngestDev& ingest_dev(int device) {
    std::lock_guard<std::mutex> lk(g_ingest_mu);
    auto& p = g_ingest[device];
    if (!p) {
        int ndev = 0;
        HIPCHK(hipGetDeviceCount(&ndev));
        REQUIRE(device >= 0 && device < ndev, "device ordinal out of range");
        p.reset(new IngestDev());
        DeviceScope dev_scope_((device));
        GateLock gate_(capture_gate());
        HIPCHK(hipStreamCreateWithFlags(&p->s, hipStreamNonBlocking));
        p->leaves = dalloc<int2>(128, p->owned);
    }
    return *p;
}

template <typename T>
T* grow(T*& ptr, size_t& cap, size_t n, std::vector<void*>& owned) {
    if (n > cap) {
        // the caller holds the device mutex and its last call synchronised the stream, so
        // the old buffer is idle: free it rather than keep every superseded size alive
        dfree(ptr, owned);
        cap = n + n / 2 + 1024;
        ptr = dalloc<T>(cap, owned);
    }
    return ptr;
}

// numpy FLOAT_pairwise_sum tree of one block of n elements: leaves in order
void pw_leaves(int64_t off, int64_t n, std::vector<int2>& out) {
    if (n <= 128) {
        out.push_back(make_int2((int)off, (int)n));
        return;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    pw_leaves(off, n2, out);
    pw_leaves(off + n2, n - n2, out);
}
// the same tree combining the leaf sums (float32 adds, left + right)
float pw_combine(int64_t n, const float*& leaf) {
    if (n <= 128) return *leaf++;
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    const float a = pw_combine(n2, leaf);
    const float b = pw_combine(n - n2, leaf);
    return a + b;
}

// numpy: np.mean(np.square(mono(pcm) / 32768)) as float32, bit for bit
float ingest_mean_square(IngestDev& g, const int16_t* pcm, int64_t n, int ch) {
    const int64_t full = n / 8192, tail = n % 8192;
    std::vector<int2> lv;
    if (tail) pw_leaves(0, tail, lv);
    REQUIRE(lv.size() <= 128, "tail leaves");
    const size_t ns = (size_t)full + lv.size();
    grow(g.sums, g.sums_cap, ns + 1, g.owned);
    if (!lv.empty()) HIPCHK(hipMemcpyAsync(g.leaves, lv.data(), lv.size() * sizeof(int2), hipMemcpyHostToDevice, g.s));
    launch_ingest_sumsq(pcm, ch, (int)full, g.leaves, (int)lv.size(), g.sums, g.sums + full, g.s);
    HIPCHK(hipGetLastError());
    std::vector<float> h(ns);
    if (ns) HIPCHK(hipMemcpyAsync(h.data(), g.sums, ns * 4, hipMemcpyDeviceToHost, g.s));
    HIPCHK(hipStreamSynchronize(g.s));
    // np.add.reduce: the 8192-element blocks' pairwise sums added in order
    float acc = 0.f;
    for (int64_t b = 0; b < full; ++b) acc = b == 0 ? h[0] : acc + h[b];
    if (tail) {
        const float* p = h.data() + full;
        const float t = pw_combine(tail, p);
        acc = full ? acc + t : t;
    }
    return acc / (float)n;
}

int64_t upfirdn_output_len(int64_t len_h, int64_t n_in, int64_t up, int64_t down) {
    const int64_t nt = (n_in + (len_h + ((up - len_h % up) % up)) / up - 1) * up;
    return nt / down + (nt % down ? 1 : 0);
}

}  // namespace

// ------------------------------ decode sessions ------------------------------
// Continuous batching (osw_session_*, include/osw.h): c->B window slots, `beam` decoder rows
// each (rows slot*beam .. slot*beam+beam-1), per-row step counters (pos[row]), per-row prompts
// (SelState::plen, prompt rows of n_text_ctx ints).  The self-K/V cache and the cross-K/V
// keep their full-capacity layouts (ctx->kv_rows, ctx->xkv_windows), so a step may cover only
// the rows up to the highest occupied slot.  Windows are admitted between chunks of CH steps:
// their log-mel, their encoder straight into the slots' cross-K/V, then the rows' reset.
struct SessionWin {
    int64_t clip;            // ClipStore key (a private key < 0 for a window that brought its own PCM)
    std::vector<int> prefix;
    osw_session_window w;
};

// The log-mel of every clip a decode session holds windows of, computed ONCE when the clip's
// first window is added and kept on the device until the caller releases the clip
// (osw_session_release_clip) or the session ends: a long file's later windows are staged
// from it (a device-to-device copy of the window's frames and the clip's max) instead of
// re-uploading the whole clip and recomputing its log-mel per window.  One
// arena per context, first-fit spans, grown by doubling (the old contents keep their
// offsets); per-clip maxima in a slot array.  Lives as long as the context.
struct ClipStore {
    struct Clip {
        int64_t off = 0;   // first float of the clip's [nframes][n_mels] log10 mel in the arena
        int nframes = 0;
        int slot = 0;      // its max (ordered int) at maxv[slot]
        bool priv = false; // registered for one window (no caller key): released at its admission
    };
    std::map<int64_t, Clip> clips;
    int64_t next_priv = -2;
    float* arena = nullptr;
    int64_t cap = 0;                   // floats
    std::map<int64_t, int64_t> spans;  // free spans: offset -> length (coalesced)
    int* maxv = nullptr;
    int slots_cap = 0;
    std::vector<int> free_slots;
    int64_t* hdr = nullptr;            // one clip's mel launch: pcm offsets {0, n}, mel_off {off, end}, nframes
};
struct Session {
    osw_decode_opts o{};
    SelParams SP{};
    int beam = 1, W = 0, tail = 3, max_len = 448, max_tok = 445, ctx = 448;
    std::vector<int64_t> slot_tag;
    std::deque<SessionWin> queue;
    int active = 0;
    int64_t steps = 0;
};

namespace {
using osw::SelState;

ClipStore& clip_store(osw_ctx* c) {
    if (!c->cstore) {
        c->cstore = new ClipStore();
        c->cstore->hdr = dalloc<int64_t>(6, c->owned);
    }
    return *c->cstore;
}

int64_t store_alloc(osw_ctx* c, ClipStore& cs, int64_t len) {
    for (auto it = cs.spans.begin(); it != cs.spans.end(); ++it)
        if (it->second >= len) {
            const int64_t off = it->first, rest = it->second - len;
            cs.spans.erase(it);
            if (rest) cs.spans[off + len] = rest;
            return off;
        }
    // grow: a bigger arena holding the old one's contents at the same offsets
    const int64_t ncap = std::max<int64_t>(std::max<int64_t>(2 * cs.cap, cs.cap + len),
                                           (int64_t)std::max(4, c->B) * 3001 * c->d.n_mels);
    float* na = dalloc<float>((size_t)ncap, c->owned);
    if (cs.arena) {
        HIPCHK(hipMemcpyAsync(na, cs.arena, (size_t)cs.cap * 4, hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        dfree(cs.arena, c->owned);
    }
    int64_t tail_off = cs.cap, tail_len = ncap - cs.cap;
    if (!cs.spans.empty()) {
        auto last = std::prev(cs.spans.end());
        if (last->first + last->second == cs.cap) {
            tail_off = last->first;
            tail_len += last->second;
            cs.spans.erase(last);
        }
    }
    cs.arena = na;
    cs.cap = ncap;
    cs.spans[tail_off + len] = tail_len - len;
    if (tail_len == len) cs.spans.erase(tail_off + len);
    return tail_off;
}

void store_free(ClipStore& cs, int64_t off, int64_t len) {
    auto it = cs.spans.emplace(off, len).first;
    if (it != cs.spans.begin()) {
        auto prev = std::prev(it);
        if (prev->first + prev->second == off) {
            prev->second += it->second;
            cs.spans.erase(it);
            it = prev;
        }
    }
    auto next = std::next(it);
    if (next != cs.spans.end() && it->first + it->second == next->first) {
        it->second += next->second;
        cs.spans.erase(next);
    }
}

// Registers a clip: its PCM uploaded and its log-mel computed into the store (on the stream)
void store_add(osw_ctx* c, int64_t key, const int16_t* pcm, int64_t n, bool priv) {
    ClipStore& cs = clip_store(c);
    REQUIRE(n >= 0, "bad clip length");
    const int n_mels = c->d.n_mels;
    ClipStore::Clip cl;
    cl.nframes = (int)((n + 160) / 160);
    cl.priv = priv;
    cl.off = store_alloc(c, cs, (int64_t)cl.nframes * n_mels);
    if (cs.free_slots.empty()) {
        const int ncap = std::max(64, 2 * cs.slots_cap);
        int* nm = dalloc<int>(ncap, c->owned);
        if (cs.maxv) {
            HIPCHK(hipMemcpyAsync(nm, cs.maxv, (size_t)cs.slots_cap * 4, hipMemcpyDeviceToDevice, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            dfree(cs.maxv, c->owned);
        }
        for (int i = ncap - 1; i >= cs.slots_cap; --i) cs.free_slots.push_back(i);
        cs.maxv = nm;
        cs.slots_cap = ncap;
    }
    cl.slot = cs.free_slots.back();
    cs.free_slots.pop_back();
    if ((size_t)n > c->pcm_cap) {
        c->pcm_cap = (size_t)n + (size_t)n / 2 + 1;
        dfree(c->pcm, c->owned);
        c->pcm = dalloc<int16_t>(c->pcm_cap, c->owned);
    }
    if (n) HIPCHK(hipMemcpyAsync(c->pcm, pcm, (size_t)n * 2, hipMemcpyHostToDevice, c->stream));
    const int64_t h[6] = {0, n, cl.off, cl.off + (int64_t)cl.nframes * n_mels, cl.nframes, 0};
    HIPCHK(hipMemcpyAsync(cs.hdr, h, sizeof(h), hipMemcpyHostToDevice, c->stream));
    {
        Timed t(c, CL_MEL, (double)n * 2 + (double)cl.nframes * n_mels * 4);
        // (nframes as the low int of hdr[4]: little-endian)
        launch_mel(c->pcm, cs.hdr, cs.hdr + 2, (const int*)(cs.hdr + 4), 1, cl.nframes, c->tw400, c->hann, c->flo,
                   c->fcnt, c->foff, c->fw, n_mels, cs.arena, cs.maxv + cl.slot, c->stream);
        HIPCHK(hipGetLastError());
    }
    cs.clips[key] = cl;
}

void store_release(osw_ctx* c, int64_t key) {
    if (!c->cstore) return;
    ClipStore& cs = *c->cstore;
    auto it = cs.clips.find(key);
    if (it == cs.clips.end()) return;
    store_free(cs, it->second.off, (int64_t)it->second.nframes * c->d.n_mels);
    cs.free_slots.push_back(it->second.slot);
    cs.clips.erase(it);
}

void store_clear(osw_ctx* c) {
    if (!c->cstore) return;
    std::vector<int64_t> keys;
    for (auto& kv : c->cstore->clips) keys.push_back(kv.first);
    for (int64_t k : keys) store_release(c, k);
}

void session_begin(osw_ctx* c, const osw_decode_opts* o) {
    REQUIRE(o, "null decode options");
    REQUIRE(!c->sess, "a decode session is already open on this context");
    REQUIRE(!(o->temperature > 0.f), "decode sessions decode at temperature 0 (greedy or beam search)");
    const osw_dims& d = c->d;
    const int V = d.n_vocab;
    REQUIRE(V <= SEL_SPLIT * 4096, "vocabulary too large for the selection kernels");
    auto S = std::make_unique<Session>();
    S->o = *o;
    S->beam = std::max(1, o->beam_size);
    REQUIRE(S->beam <= 5, "decode sessions hold beam_size <= 5 (5 decoder rows per window slot)");
    S->W = c->B;
    S->ctx = d.n_text_ctx;
    S->tail = 3 + (o->without_timestamps ? 1 : 0);
    S->max_len = std::min(o->max_length > 0 ? o->max_length : d.n_text_ctx, d.n_text_ctx);
    REQUIRE(S->tail < S->max_len, "prompt longer than max_length");
    S->max_tok = std::max(1, S->max_len - S->tail);
    std::vector<unsigned> mask((V + 31) / 32, 0u);
    for (int i = 0; i < o->n_suppress; ++i) {
        const int t = o->suppress_tokens[i];
        if (t >= 0 && t < V) mask[t >> 5] |= 1u << (t & 31);
    }
    SelParams& SP = S->SP;
    SP.prompt_len = S->tail; SP.sot_pos = 0; SP.lang_pos = 1; SP.max_length = S->max_len;
    SP.pstride = S->ctx; SP.tail = S->tail;
    SP.V = V; SP.eot = o->eot; SP.no_speech = o->no_speech; SP.no_ts = o->no_timestamps; SP.tb = o->timestamp_begin;
    SP.blank = o->blank; SP.first_lang = o->first_lang; SP.n_langs = o->n_langs;
    SP.suppress_blank = o->suppress_blank; SP.with_ts = o->without_timestamps ? 0 : 1;
    SP.max_init_ts = o->max_initial_timestamp_index;
    SP.beam = S->beam;
    SP.num_hyp = std::max(1, o->num_hypotheses);
    SP.max_cand = std::max(1, (int)std::lround(S->beam * (o->patience > 0.f ? o->patience : 1.f)));
    SP.length_penalty = o->length_penalty;
    SP.inv_temp = 0.f;
    HIPCHK(hipMemcpyAsync(c->seed_d, &o->seed, 8, hipMemcpyHostToDevice, c->stream));
    SP.seed = c->seed_d;
    SP.budget = c->budget;
    SP.pos_row = 1;
    S->o.suppress_tokens = nullptr;  // (copied into the mask)
    S->o.prefix_tokens = nullptr;
    S->o.language_tokens = nullptr;
    S->o.token_budget = nullptr;
    const int R = S->W * S->beam;
    std::vector<SelState> st(R);
    for (auto& q : st) q = SelState{}, q.done = 1;
    HIPCHK(hipMemcpyAsync(c->supmask, mask.data(), mask.size() * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->sel, st.data(), (size_t)R * sizeof(SelState), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemsetAsync(c->pos, 0, (size_t)R * 4, c->stream));
    HIPCHK(hipMemsetAsync(c->cur_tok, 0, (size_t)R * 4, c->stream));
    HIPCHK(hipMemsetAsync(c->budget, 0, (size_t)R * 4, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    S->slot_tag.assign(S->W, -1);
    c->row_pos = true;
    c->kv_rows = c->R;
    c->xkv_windows = c->B;
    c->sess = S.release();
}

void session_end(osw_ctx* c) {
    store_clear(c);
    delete c->sess;
    c->sess = nullptr;
    c->row_pos = false;
    c->kv_rows = 0;
    c->xkv_windows = 0;
    c->n_encoded = 0;
}

void session_add(osw_ctx* c, const int16_t* pcm, const int64_t* offsets, int n, const osw_session_window* w) {
    Session* S = c->sess;
    REQUIRE(S, "no decode session open");
    REQUIRE(pcm && offsets && w && n >= 0, "null argument");
    // every window is checked before any is queued or any clip registered
    ClipStore& cs = clip_store(c);
    std::map<int64_t, int64_t> fresh;  // caller keys registered by this call -> window index
    for (int i = 0; i < n; ++i) {
        REQUIRE(offsets[i + 1] >= offsets[i], "offsets must not decrease");
        REQUIRE(w[i].segment_size >= 1 && w[i].seek >= 0, "empty window");
        REQUIRE(w[i].n_prefix >= 0 && (w[i].n_prefix == 0 || w[i].prefix), "bad prefix");
        REQUIRE(w[i].n_prefix + S->tail < S->max_len, "prompt longer than max_length");
        int64_t samples = offsets[i + 1] - offsets[i];
        if (w[i].clip >= 0) {
            auto it = cs.clips.find(w[i].clip);
            if (it != cs.clips.end()) {
                samples = -1;
                REQUIRE(w[i].seek < it->second.nframes, "window seek out of range");
            } else if (fresh.count(w[i].clip)) {
                samples = offsets[fresh[w[i].clip] + 1] - offsets[fresh[w[i].clip]];
            } else {
                fresh[w[i].clip] = i;
            }
        }
        // (log_mel's frame count: one frame per 160 samples, plus one)
        if (samples >= 0) REQUIRE(w[i].seek < (int)((samples + 160) / 160), "window seek out of range");
    }
    for (int i = 0; i < n; ++i) {
        SessionWin q;
        if (w[i].clip >= 0) {
            if (!cs.clips.count(w[i].clip)) store_add(c, w[i].clip, pcm + offsets[i], offsets[i + 1] - offsets[i], false);
            q.clip = w[i].clip;
        } else {
            q.clip = cs.next_priv--;
            store_add(c, q.clip, pcm + offsets[i], offsets[i + 1] - offsets[i], true);
        }
        q.prefix.assign(w[i].prefix, w[i].prefix + w[i].n_prefix);
        q.w = w[i];
        q.w.prefix = nullptr;
        S->queue.push_back(std::move(q));
    }
}

void session_admit(osw_ctx* c, int refill_min) {
    Session* S = c->sess;
    std::vector<int> free_slots;
    for (int i = 0; i < S->W; ++i)
        if (S->slot_tag[i] < 0) free_slots.push_back(i);
    const int queued = (int)S->queue.size();
    if (!queued || free_slots.empty()) return;
    if (S->active > 0 && (int)free_slots.size() < std::min(std::max(1, refill_min), queued)) return;
    const int k = std::min((int)free_slots.size(), queued);
    // the admitted windows' frames, staged from their clips' resident log-mel as k "clips"
    // (window i = its frames [seek, seek + min(segment, frames - seek)) and its clip's max), so
    // encode() sees the layout log_mel() writes
    ClipStore& cs = clip_store(c);
    const int n_mels = c->d.n_mels;
    if (k > c->clips_cap) {
        const int cap = std::max(k, 2 * c->clips_cap);
        dfree(c->offsets, c->owned);
        dfree(c->mel_off_d, c->owned);
        dfree(c->nframes_d, c->owned);
        dfree(c->clip_max, c->owned);
        c->offsets = dalloc<int64_t>(cap + 1, c->owned);
        c->mel_off_d = dalloc<int64_t>(cap + 1, c->owned);
        c->nframes_d = dalloc<int>(cap, c->owned);
        c->clip_max = dalloc<int>(cap, c->owned);
        c->clips_cap = cap;
    }
    c->nframes.assign(k, 0);
    c->mel_off.assign(k + 1, 0);
    std::vector<int64_t> src_off(k);
    std::vector<int> src_slot(k);
    for (int i = 0; i < k; ++i) {
        const SessionWin& q = S->queue[i];
        const ClipStore::Clip& cl = cs.clips.at(q.clip);
        const int len = std::max(1, std::min(std::min(q.w.segment_size, N_FR), cl.nframes - q.w.seek));
        c->nframes[i] = len;
        c->mel_off[i + 1] = c->mel_off[i] + (int64_t)len * n_mels;
        src_off[i] = cl.off + (int64_t)q.w.seek * n_mels;
        src_slot[i] = cl.slot;
    }
    if ((size_t)c->mel_off[k] > c->logmel_cap) {
        c->logmel_cap = (size_t)c->mel_off[k] + (size_t)c->mel_off[k] / 2;
        dfree(c->logmel, c->owned);
        c->logmel = dalloc<float>(c->logmel_cap, c->owned);
    }
    for (int i = 0; i < k; ++i) {
        HIPCHK(hipMemcpyAsync(c->logmel + c->mel_off[i], cs.arena + src_off[i],
                              (size_t)(c->mel_off[i + 1] - c->mel_off[i]) * 4, hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(c->clip_max + i, cs.maxv + src_slot[i], 4, hipMemcpyDeviceToDevice, c->stream));
    }
    HIPCHK(hipMemcpyAsync(c->mel_off_d, c->mel_off.data(), (k + 1) * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->nframes_d, c->nframes.data(), k * 4, hipMemcpyHostToDevice, c->stream));
    c->n_clips = k;
    const int ps = 3 + S->ctx;
    std::vector<osw_window> wins(k);
    std::vector<int> slots(k), pack((size_t)k * ps, 0);
    for (int i = 0; i < k; ++i) {
        const SessionWin& q = S->queue[i];
        const int slot = free_slots[i];
        wins[i] = osw_window{i, 0, q.w.segment_size};
        slots[i] = slot;
        int* e = &pack[(size_t)i * ps];
        const int np = (int)q.prefix.size();
        e[0] = slot;
        e[1] = np + S->tail;
        e[2] = q.w.token_budget;
        for (int j = 0; j < np; ++j) e[3 + j] = q.prefix[j];
        e[3 + np] = S->o.sot;
        e[3 + np + 1] = q.w.language_token;  // -1: detect
        e[3 + np + 2] = S->o.task_token;
        if (S->o.without_timestamps) e[3 + np + 3] = S->o.no_timestamps;
    }
    encode(c, wins.data(), k, slots.data());
    for (int i = 0; i < k; ++i) S->slot_tag[free_slots[i]] = S->queue[i].w.tag;
    HIPCHK(hipMemcpyAsync(c->refill_pack, pack.data(), pack.size() * 4, hipMemcpyHostToDevice, c->stream));
    launch_session_rows(c->refill_pack, k, ps, S->beam, S->ctx, S->ctx, c->prompt, c->budget, c->cur_tok, c->pos,
                        c->sel, S->beam > 1 ? c->anc : nullptr, S->beam > 1 ? c->bwin : nullptr, c->stream);
    HIPCHK(hipGetLastError());
    for (int i = 0; i < k; ++i) {
        if (S->queue.front().clip < 0) store_release(c, S->queue.front().clip);  // (its frames were staged)
        S->queue.pop_front();
    }
    S->active += k;
}

// returns the number of finished windows written to r / tags
int session_step(osw_ctx* c, int max_chunks, int refill_min, osw_window_result* r, int64_t* tags, int cap) {
    Session* S = c->sess;
    REQUIRE(S, "no decode session open");
    REQUIRE(r && r->tokens && r->n_tokens && r->sum_logprob && r->no_speech_prob && r->language && tags,
            "null result argument");
    REQUIRE(cap >= S->W, "cap must hold every slot (max_batch)");
    // OSW_SESSION_CHUNK: decoder steps between admission points.  4 since round 6 (config 5
    // 177-179 vs 171-172 calls/s, REST mixed continuous 74-75 vs 73 calls/s with p50 117-122
    // vs 136-141 ms: profiles/r06_zcd_session_chunk_ab.txt); 8 before (decode()'s chunk)
    static const int CH = [] {
        const char* e = getenv("OSW_SESSION_CHUNK");
        return e ? std::max(1, std::min(64, atoi(e))) : 4;
    }();
    const int beam = S->beam;
    int done = 0;
    if (max_chunks == 0) {  // admission only: the queued windows' encoder, waited for
        session_admit(c, refill_min);
        HIPCHK(hipStreamSynchronize(c->stream));
        return 0;
    }
    for (int chunk = 0; chunk < max_chunks && done == 0; ++chunk) {
        session_admit(c, refill_min);
        if (S->active == 0) break;
        int hi = 0;
        for (int i = 0; i < S->W; ++i)
            if (S->slot_tag[i] >= 0) hi = i + 1;
        if (hi > 4) hi = std::min(S->W, (hi + 3) / 4 * 4);  // (fewer graph shapes; idle slots' rows are finished)
        const int nb = hi * beam;
        const SelParams& SP = S->SP;
        auto one_step = [&] {
            decoder_step(c, nb, beam, beam > 1, nullptr);
            launch_select(c->logits, nb, c->pos, SP, c->prompt, c->supmask, c->sel, c->cur_tok, c->tokens, S->max_tok,
                          c->selp, c->sel_arrive, beam == 1, c->bcand, c->stream);
            if (beam > 1)
                launch_beam(c->logits, hi, c->pos, SP, c->supmask, c->sel, c->selp, c->bcand, c->tokens, c->anc, S->ctx,
                            c->bwin, c->btok, c->cur_tok, S->max_tok, c->sel_arrive, c->stream);
        };
        if (c->use_graph && !c->prof_eager) {
            int32_t lp_bits;
            std::memcpy(&lp_bits, &SP.length_penalty, 4);
            // (the -2 tail keeps session keys apart from decode()'s and the refill's)
            const std::vector<int64_t> key = {nb, S->tail, 0, S->max_len, S->o.eot, S->o.no_speech, S->o.no_timestamps,
                                              S->o.timestamp_begin, S->o.blank, S->o.first_lang, S->o.n_langs,
                                              S->o.suppress_blank, S->o.without_timestamps,
                                              S->o.max_initial_timestamp_index, beam, SP.num_hyp, SP.max_cand, lp_bits,
                                              beam, 0, 1, -2, CH};
            hipGraphExec_t ge = decode_graph(c, key, one_step, CH);
            trace_graph(c, "launch");
            HIPCHK(hipGraphLaunch(ge, c->stream));
        } else {
            for (int i = 0; i < CH; ++i) one_step();
        }
        HIPCHK(hipGetLastError());
        S->steps += CH;
        std::vector<SelState> st(nb);
        std::vector<BeamWin> bw(beam > 1 ? hi : 0);
        HIPCHK(hipMemcpyAsync(st.data(), c->sel, (size_t)nb * sizeof(SelState), hipMemcpyDeviceToHost, c->stream));
        if (beam > 1)
            HIPCHK(hipMemcpyAsync(bw.data(), c->bwin, (size_t)hi * sizeof(BeamWin), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        std::vector<int> fin;
        for (int i = 0; i < hi; ++i)
            if (S->slot_tag[i] >= 0 && (beam > 1 ? bw[i].done : st[i].done)) fin.push_back(i);
        if (fin.empty()) continue;
        // the finished windows' tokens: beam -> the best hypothesis per window (btok),
        // greedy -> the row's picks (tokens)
        std::vector<int> toks((size_t)hi * S->max_tok);
        HIPCHK(hipMemcpyAsync(toks.data(), beam > 1 ? c->btok : c->tokens, toks.size() * 4, hipMemcpyDeviceToHost,
                              c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        for (int slot : fin) {
            const SelState& q = st[(size_t)slot * beam];
            const int n0 = beam > 1 ? bw[slot].best_len : q.n_sampled;
            const int n = std::min(n0, std::min(S->max_tok, r->max_tokens));
            r->n_tokens[done] = n;
            for (int j = 0; j < n; ++j) r->tokens[(size_t)done * r->max_tokens + j] = toks[(size_t)slot * S->max_tok + j];
            r->sum_logprob[done] = beam > 1 ? bw[slot].best_raw : q.sum_lp;
            r->no_speech_prob[done] = q.nsp;
            r->language[done] = q.lang;
            tags[done] = S->slot_tag[slot];
            S->slot_tag[slot] = -1;
            --S->active;
            ++done;
        }
    }
    c->pf.decode_steps = S->steps;
    return done;
}
}  // namespace

// ============================== C ABI =======================================
extern "C" {

const char* osw_version(void) { return "osw-hip 0.1 gfx950"; }
const char* osw_last_error(void) { return g_err.c_str(); }

int osw_device_count(int32_t* out) {
    return guard([&] {
        int n = 0;
        HIPCHK(hipGetDeviceCount(&n));
        *out = n;
    });
}

void make_streams(osw_ctx* c) {
    // measured: 4651 / 4625 vs 4748 / 4743 audio-s/s (12 steps, baton on), so opt-in only
    const char* ep = std::getenv("OSW_ENC_PRIO");
    if (!ep || ep[0] != '1') {
        HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        return;
    }
    int lo = 0, hi = 0;  // least and greatest priority (greatest is numerically lowest)
    HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIPCHK(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi));
    HIPCHK(hipStreamCreateWithPriority(&c->enc_stream, hipStreamNonBlocking, lo));
    HIPCHK(hipEventCreateWithFlags(&c->enc_in, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&c->enc_out, hipEventDisableTiming));
}

void destroy_streams(osw_ctx* c) {
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->enc_stream) (void)hipStreamDestroy(c->enc_stream);
    if (c->enc_in) (void)hipEventDestroy(c->enc_in);
    if (c->enc_out) (void)hipEventDestroy(c->enc_out);
}

int osw_create(const osw_dims* dims, int32_t device, int32_t max_batch, osw_ctx** out) {
    osw_ctx* c = nullptr;
    int rc = guard([&] {
        REQUIRE(dims && out, "null argument");
        REQUIRE(max_batch >= 1 && max_batch <= 1024, "max_batch out of range");
        REQUIRE(dims->n_audio_state % 128 == 0 && dims->n_text_state % 128 == 0, "model width must be a multiple of 128");
        REQUIRE(dims->n_audio_state / dims->n_audio_head == 64 && dims->n_text_state / dims->n_text_head == 64,
                "head_dim must be 64");
        REQUIRE(dims->n_audio_ctx == T_ENC, "n_audio_ctx must be 1500");
        REQUIRE(dims->n_text_ctx <= 448, "n_text_ctx must be <= 448");
        REQUIRE(dims->n_audio_state == dims->n_text_state, "encoder and decoder width must match");
        REQUIRE(dims->n_audio_state <= 1280, "model width > 1280 unsupported");
        int ndev = 0;
        HIPCHK(hipGetDeviceCount(&ndev));
        REQUIRE(device >= 0 && device < ndev, "device ordinal out of range");
        GateLock gate_(capture_gate());  // streams, allocations, kernel attributes
        c = new osw_ctx();
        c->device = device;
        c->d = *dims;
        c->B = max_batch;
        c->R = max_batch * 5;  // room for the reference's beam_size = 5 at full batch
        c->C1 = (dims->n_mels + 63) / 64 * 64;
        if (const char* e = std::getenv("OSW_NO_GRAPH")) c->use_graph = !(e[0] == '1');
        // OSW_BATON_MIN_WINDOWS=n: encoders below n windows skip the baton (0: never skip)
        if (const char* e = std::getenv("OSW_BATON_MIN_WINDOWS")) c->baton_min = atoi(e);
        DeviceScope dev_scope_((device));
        prepare_gemm_kernels();  // no kernel attribute is set lazily beside other lanes' launches
        make_streams(c);
        const char* eb = std::getenv("OSW_ENC_BATON");
        if (!eb || eb[0] != '0') {
            c->baton = std::make_shared<EncBaton>();
            HIPCHK(hipEventCreateWithFlags(&c->baton->ev, hipEventDisableTiming));
        }
        build_weight_table(c);
        setup_mel(c);
        setup_workspace(c);
        HIPCHK(hipStreamSynchronize(c->stream));
        *out = c;
    });
    if (rc != OSW_OK && c) {
        GateLock gate_(capture_gate());
        for (void* p : c->owned) (void)hipFree(p);
        destroy_streams(c);
        delete c;
    }
    return rc;
}

int osw_create_sibling(osw_ctx* parent, int32_t max_batch, osw_ctx** out) {
    osw_ctx* c = nullptr;
    int rc = guard([&] {
        REQUIRE(parent && out, "null argument");
        REQUIRE(max_batch >= 1 && max_batch <= 1024, "max_batch out of range");
        std::lock_guard<std::mutex> lk(parent->mu);
        REQUIRE(parent->finalized, "parent context weights not finalized");
        GateLock gate_(capture_gate());
        c = new osw_ctx();
        c->device = parent->device;
        c->d = parent->d;
        c->B = max_batch;
        c->R = max_batch * 5;
        c->C1 = parent->C1;
        c->use_graph = parent->use_graph;
        c->baton_min = parent->baton_min;
        DeviceScope dev_scope_((c->device));
        make_streams(c);
        c->w = parent->w;          // same device pointers
        c->arena = parent->arena;  // keeps the weights alive past the parent's destroy
        c->baton = parent->baton;
        c->sibling = true;
        c->finalized = true;
        setup_mel(c);
        setup_workspace(c);
        HIPCHK(hipStreamSynchronize(c->stream));
        *out = c;
    });
    if (rc != OSW_OK && c) {
        GateLock gate_(capture_gate());
        for (void* p : c->owned) (void)hipFree(p);
        destroy_streams(c);
        delete c;
    }
    return rc;
}

int osw_destroy(osw_ctx* c) {
    if (!c) return OSW_OK;
    return guard([&] {
        {
            std::lock_guard<std::mutex> lk(c->mu);
            DeviceScope dev_scope_((c->device));
            HIPCHK(hipStreamSynchronize(c->stream));
            GateLock gate_(capture_gate());
            for (auto& e : c->evs) { (void)hipEventDestroy(e.a); (void)hipEventDestroy(e.b); }
            for (auto e : c->ev_free) (void)hipEventDestroy(e);
            for (auto& kv : c->dgraphs) (void)hipGraphExecDestroy(kv.second.first);
            delete c->sess;
            c->sess = nullptr;
            delete c->cstore;
            c->cstore = nullptr;
            for (void* p : c->owned) (void)hipFree(p);
            if (c->done_host) (void)hipHostFree(c->done_host);
            destroy_streams(c);
            c->arena.reset();
        }
        delete c;
    });
}

int osw_set_weight(osw_ctx* c, const char* name, const void* host, int64_t nbytes) {
    return guard([&] {
        REQUIRE(c && name && host, "null argument");
        std::lock_guard<std::mutex> lk(c->mu);
        REQUIRE(!c->sibling, "sibling contexts share their parent's weights (read-only)");
        DeviceScope dev_scope_((c->device));
        GateLock gate_(capture_gate());  // weight upload (a model loading while another serves)
        Tensor& t = W(c, name);
        const std::string nm(name);
        if (nm == "enc.conv1.w" && c->C1 != c->d.n_mels) {
            const int64_t De = c->d.n_audio_state, M = c->d.n_mels;
            REQUIRE(nbytes == De * 3 * M * 2, "enc.conv1.w: wrong byte count");
            std::vector<uint16_t> pad((size_t)De * 3 * c->C1, 0);
            const uint16_t* src = (const uint16_t*)host;
            for (int64_t o = 0; o < De; ++o)
                for (int k = 0; k < 3; ++k)
                    std::memcpy(&pad[(o * 3 + k) * c->C1], &src[(o * 3 + k) * M], M * 2);
            HIPCHK(hipMemcpyAsync(t.ptr, pad.data(), pad.size() * 2, hipMemcpyHostToDevice, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));  // before `pad` goes
        } else {
            REQUIRE(nbytes == t.numel * (t.f16 ? 2 : 4), "tensor " + nm + ": wrong byte count");
            HIPCHK(hipMemcpyAsync(t.ptr, host, nbytes, hipMemcpyHostToDevice, c->stream));
        }
        pack_frag(c, nm);
        HIPCHK(hipStreamSynchronize(c->stream));
        t.set = true;
    });
}

int osw_get_weight(osw_ctx* c, const char* name, void* host, int64_t nbytes) {
    return guard([&] {
        REQUIRE(c && name && host, "null argument");
        std::lock_guard<std::mutex> lk(c->mu);
        DeviceScope dev_scope_((c->device));
        Tensor& t = W(c, name);
        REQUIRE(nbytes == t.numel * (t.f16 ? 2 : 4), std::string("tensor ") + name + ": wrong byte count");
        HIPCHK(hipMemcpyAsync(host, t.ptr, nbytes, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    });
}

int osw_init_weight_uniform(osw_ctx* c, const char* name, uint64_t seed, int64_t stream, float scale, float offset,
                            int64_t zero_lo, int64_t zero_hi) {
    return guard([&] {
        REQUIRE(c && name, "null argument");
        std::lock_guard<std::mutex> lk(c->mu);
        REQUIRE(!c->sibling, "sibling contexts share their parent's weights (read-only)");
        DeviceScope dev_scope_((c->device));
        Tensor& t = W(c, name);
        REQUIRE(!(std::string(name) == "enc.conv1.w" && c->C1 != c->d.n_mels),
                "enc.conv1.w needs osw_set_weight when n_mels is not a multiple of 64");
        launch_init_uniform(t.ptr, t.f16, t.numel, hash_stream_key(seed, stream), scale, offset, zero_lo, zero_hi,
                            c->stream);
        HIPCHK(hipGetLastError());
        pack_frag(c, name);
        HIPCHK(hipStreamSynchronize(c->stream));
        t.set = true;
    });
}

int osw_finalize(osw_ctx* c) {
    return guard([&] {
        REQUIRE(c, "null ctx");
        std::lock_guard<std::mutex> lk(c->mu);
        std::string missing;
        for (auto& kv : c->w)
            if (!kv.second.set) missing += kv.first + " ";
        REQUIRE(missing.empty(), "missing tensors: " + missing);
        c->finalized = true;
    });
}

int osw_log_mel(osw_ctx* c, const int16_t* pcm, const int64_t* offsets, int32_t n_clips, int32_t pcm_on_device,
                int32_t* n_frames) {
    return guard([&] {
        REQUIRE(c, "null ctx");
        std::lock_guard<std::mutex> lk(c->mu);
        DeviceScope dev_scope_((c->device));
        log_mel(c, pcm, offsets, n_clips, pcm_on_device, n_frames);
        HIPCHK(hipStreamSynchronize(c->stream));
        resolve_events(c);
    });
}

int osw_get_mel(osw_ctx* c, int32_t clip, float* out, int64_t out_floats) {
    return guard([&] {
        REQUIRE(c && out, "null argument");
        std::lock_guard<std::mutex> lk(c->mu);
        DeviceScope dev_scope_((c->device));
        REQUIRE(clip >= 0 && clip < c->n_clips, "clip out of range");
        const int nf = c->nframes[clip];
        const int64_t n = (int64_t)nf * c->d.n_mels;
        REQUIRE(out_floats >= n, "output buffer too small");
        std::vector<void*> tmp_owned;  // (dalloc / dfree take the capture gate)
        float* tmp = dalloc<float>((size_t)n, tmp_owned);
        launch_mel_normalize(c->logmel, c->mel_off[clip], nf, c->d.n_mels, c->clip_max, clip, tmp, c->stream);
        hipError_t e = hipMemcpyAsync(out, tmp, n * 4, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        dfree(tmp, tmp_owned);
        HIPCHK(e);
    });
}

int osw_encode_windows(osw_ctx* c, const osw_window* windows, int32_t n) {
    return guard([&] {
        REQUIRE(c && windows, "null argument");
        std::lock_guard<std::mutex> lk(c->mu);
        REQUIRE(!c->sess, "a decode session is open on this context (osw_session_end first)");
        DeviceScope dev_scope_((c->device));
        LaneCall call_(c);
        encode(c, windows, n);
        HIPCHK(hipStreamSynchronize(c->stream));
        resolve_events(c);
    });
}

int osw_get_encoder_output(osw_ctx* c, int32_t window, float* out, int64_t out_floats) {
    return guard([&] {
        REQUIRE(c && out, "null argument");
        std::lock_guard<std::mutex> lk(c->mu);
        DeviceScope dev_scope_((c->device));
        REQUIRE(window >= 0 && window < c->n_encoded, "window out of range");
        const int64_t n = (int64_t)T_ENC * c->d.n_audio_state;
        REQUIRE(out_floats >= n, "output buffer too small");
        std::vector<_Float16> tmp(n);
        HIPCHK(hipMemcpyAsync(tmp.data(), c->E + window * n, n * 2, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        for (int64_t i = 0; i < n; ++i) out[i] = (float)tmp[i];
    });
}

int osw_decode_windows(osw_ctx* c, int32_t n, const osw_decode_opts* opts, osw_window_result* res) {
    return guard([&] {
        REQUIRE(c, "null ctx");
        std::lock_guard<std::mutex> lk(c->mu);
        REQUIRE(!c->sess, "a decode session is open on this context (osw_session_end first)");
        DeviceScope dev_scope_((c->device));
        LaneCall call_(c);
        decode(c, n, opts, res);
        resolve_events(c);
    });
}

int osw_transcribe_batch(osw_ctx* c, const int16_t* pcm, const int64_t* offsets, int32_t n_clips,
                         int32_t pcm_on_device, const osw_decode_opts* opts, osw_window_result* res) {
    return guard([&] {
        REQUIRE(c, "null ctx");
        std::lock_guard<std::mutex> lk(c->mu);
        REQUIRE(!c->sess, "a decode session is open on this context (osw_session_end first)");
        DeviceScope dev_scope_((c->device));
        REQUIRE(n_clips >= 1 && n_clips <= c->B, "n_clips out of range");
        LaneCall call_(c);
        log_mel(c, pcm, offsets, n_clips, pcm_on_device, nullptr);
        std::vector<osw_window> wins(n_clips);
        for (int i = 0; i < n_clips; ++i)
            wins[i] = osw_window{i, 0, std::max(1, std::min(N_FR, c->nframes[i] - 1))};
        encode(c, wins.data(), n_clips);
        decode(c, n_clips, opts, res);
        resolve_events(c);
    });
}

int osw_transcribe_refill(osw_ctx* c, const int16_t* pcm, const int64_t* offsets, int32_t n_clips,
                          int32_t pcm_on_device, const osw_decode_opts* opts, osw_window_result* res,
                          int32_t refill_min) {
    return guard([&] {
        REQUIRE(c, "null ctx");
        std::lock_guard<std::mutex> lk(c->mu);
        REQUIRE(!c->sess, "a decode session is open on this context (osw_session_end first)");
        DeviceScope dev_scope_((c->device));
        REQUIRE(n_clips >= 1, "n_clips out of range");
        LaneCall call_(c);
        log_mel(c, pcm, offsets, n_clips, pcm_on_device, nullptr);
        decode_refill(c, n_clips, opts, res, refill_min);
        resolve_events(c);
    });
}

int osw_session_begin(osw_ctx* c, const osw_decode_opts* opts) {
    return guard([&] {
        REQUIRE(c, "null ctx");
        std::lock_guard<std::mutex> lk(c->mu);
        DeviceScope dev_scope_((c->device));
        session_begin(c, opts);
    });
}

int osw_session_add(osw_ctx* c, const int16_t* pcm, const int64_t* offsets, int32_t n,
                    const osw_session_window* windows) {
    return guard([&] {
        REQUIRE(c, "null ctx");
        std::lock_guard<std::mutex> lk(c->mu);
        session_add(c, pcm, offsets, n, windows);
    });
}

int osw_session_step(osw_ctx* c, int32_t max_chunks, int32_t refill_min, osw_window_result* res, int64_t* tags_out,
                     int32_t cap, int32_t* n_done, int32_t* n_active, int32_t* n_queued) {
    return guard([&] {
        REQUIRE(c && n_done && n_active && n_queued, "null argument");
        std::lock_guard<std::mutex> lk(c->mu);
        DeviceScope dev_scope_((c->device));
        LaneCall call_(c);
        *n_done = session_step(c, std::max(0, max_chunks), refill_min, res, tags_out, cap);
        *n_active = c->sess->active;
        *n_queued = (int32_t)c->sess->queue.size();
        resolve_events(c);
    });
}

int osw_session_release_clip(osw_ctx* c, int64_t clip) {
    return guard([&] {
        REQUIRE(c, "null ctx");
        std::lock_guard<std::mutex> lk(c->mu);
        REQUIRE(c->sess, "no decode session open");
        REQUIRE(clip >= 0, "clip keys are >= 0");
        for (const SessionWin& q : c->sess->queue)
            REQUIRE(q.clip != clip, "a queued window still reads this clip");
        store_release(c, clip);
    });
}

int osw_session_end(osw_ctx* c) {
    return guard([&] {
        REQUIRE(c, "null ctx");
        std::lock_guard<std::mutex> lk(c->mu);
        DeviceScope dev_scope_((c->device));
        HIPCHK(hipStreamSynchronize(c->stream));
        session_end(c);
    });
}

int osw_encoder_layer_debug(osw_ctx* c, int32_t layer, const float* x, float* y, int32_t T) {
    return guard([&] {
        REQUIRE(c && x && y, "null argument");
        std::lock_guard<std::mutex> lk(c->mu);
        DeviceScope dev_scope_((c->device));
        REQUIRE(c->finalized, "weights not finalized");
        REQUIRE(T == T_ENC, "T must be 1500");
        REQUIRE(layer >= 0 && layer < c->d.n_audio_layer, "layer out of range");
        const int64_t n = (int64_t)T * c->d.n_audio_state;
        HIPCHK(hipMemcpyAsync(c->X, x, n * 4, hipMemcpyHostToDevice, c->stream));
        encoder_layer(c, layer, 1);
        HIPCHK(hipMemcpyAsync(y, c->X, n * 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        resolve_events(c);
    });
}

int osw_debug_gemm(osw_ctx* c, int32_t M, int32_t N, int32_t K, int32_t variant, const void* A, const void* Wt,
                   float* C, int32_t iters, float* ms) {
    return guard([&] {
        REQUIRE(c && A && Wt && C && ms, "null argument");
        REQUIRE(M >= 1 && N >= 1 && K >= 64 && K % 64 == 0 && iters >= 1, "bad GEMM shape");
        REQUIRE(variant != 3 || (M <= 64 && K % 128 == 0), "skinny needs M <= 64 and K % 128 == 0");
        REQUIRE(variant < 8 || variant > 19 || variant == 11 || N % 8 == 0,
                "the 8-phase debug variants need N % 8 == 0 (their epilogues store 8-column chunks)");
        std::lock_guard<std::mutex> lk(c->mu);
        DeviceScope dev_scope_((c->device));
        GateLock gate_(capture_gate());
        std::vector<void*> tmp;
        h16* dA = dalloc<h16>((size_t)M * K, tmp);
        h16* dW = dalloc<h16>((size_t)N * K, tmp);
        float* dC = dalloc<float>((size_t)M * N, tmp);
        float* dP = variant == 3 ? dalloc<float>((size_t)skinny_ksplit(N, K) * M * N, tmp) : nullptr;
        hipEvent_t e0, e1;
        HIPCHK(hipEventCreate(&e0));
        HIPCHK(hipEventCreate(&e1));
        try {
            HIPCHK(hipMemcpyAsync(dA, A, (size_t)M * K * 2, hipMemcpyHostToDevice, c->stream));
            HIPCHK(hipMemcpyAsync(dW, Wt, (size_t)N * K * 2, hipMemcpyHostToDevice, c->stream));
            GemmArgs g = gemm_plain(dA, K, dW, nullptr, M, N, K, dC, N, EPI_F32);
            auto run = [&] {
                if (variant == 3) launch_gemm_skinny(g, dP, c->stream);
                else launch_gemm_variant(g, variant, c->stream);
            };
            run();  // warm
            HIPCHK(hipEventRecord(e0, c->stream));
            for (int i = 0; i < iters; ++i) run();
            HIPCHK(hipEventRecord(e1, c->stream));
            HIPCHK(hipGetLastError());
            HIPCHK(hipEventSynchronize(e1));
            float t = 0.f;
            HIPCHK(hipEventElapsedTime(&t, e0, e1));
            *ms = t / iters;
            HIPCHK(hipMemcpyAsync(C, dC, (size_t)M * N * 4, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
        } catch (...) {
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
            for (void* p : tmp) (void)hipFree(p);
            throw;
        }
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        for (void* p : tmp) (void)hipFree(p);
    });
}

int osw_debug_hold_capture(osw_ctx* c, int32_t hold_ms) {
    return guard([&] {
        REQUIRE(c, "null ctx");
        REQUIRE(hold_ms >= 0 && hold_ms <= 10000, "hold_ms out of range");
        std::lock_guard<std::mutex> lk(c->mu);
        DeviceScope dev_scope_((c->device));
        // exactly the locks decode_graph holds around a capture
        std::unique_lock<std::mutex> no_encoder;
        if (c->baton) no_encoder = std::unique_lock<std::mutex>(c->baton->mu);
        GateLock gate_(capture_gate());
        HIPCHK(hipStreamSynchronize(c->stream));
        hipGraph_t gr = nullptr;
        c->capturing = true;
        try {
            HIPCHK(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
            HIPCHK(hipMemsetAsync(c->done, 0, sizeof(int), c->stream));  // one captured node
            const auto t0 = std::chrono::steady_clock::now();
            while (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(hold_ms)) {
                std::this_thread::sleep_for(std::chrono::milliseconds(1));
                hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
                HIPCHK(hipStreamIsCapturing(c->stream, &st));
                REQUIRE(st == hipStreamCaptureStatusActive, "the capture was invalidated while held");
            }
            HIPCHK(hipStreamEndCapture(c->stream, &gr));
        } catch (...) {
            c->capturing = false;
            hipGraph_t junk = nullptr;
            (void)hipStreamEndCapture(c->stream, &junk);
            if (junk) (void)hipGraphDestroy(junk);
            (void)hipGetLastError();
            throw;
        }
        c->capturing = false;
        REQUIRE(gr != nullptr, "empty capture");
        hipGraphExec_t ge = nullptr;
        hipError_t e = hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
        (void)hipGraphDestroy(gr);
        HIPCHK(e);
        (void)hipGraphExecDestroy(ge);
    });
}

int osw_set_encoder_baton_min(osw_ctx* c, int32_t min_windows) {
    return guard([&] {
        REQUIRE(c, "null ctx");
        REQUIRE(min_windows >= 0, "min_windows must be >= 0");
        std::lock_guard<std::mutex> lk(c->mu);
        c->baton_min = min_windows;
    });
}

int osw_set_profiling(osw_ctx* c, int32_t enable) {
    return guard([&] {
        REQUIRE(c, "null ctx");
        std::lock_guard<std::mutex> lk(c->mu);
        REQUIRE(enable >= 0 && enable <= 2, "profiling mode must be 0, 1 or 2");
        c->prof = enable != 0;
        c->prof_eager = enable == 2;
        c->pf = osw_profile{};
    });
}

int osw_get_profile(osw_ctx* c, osw_profile* out) {
    return guard([&] {
        REQUIRE(c && out, "null argument");
        std::lock_guard<std::mutex> lk(c->mu);
        resolve_events(c);
        *out = c->pf;
    });
}

void* osw_stream(osw_ctx* c) { return c ? (void*)c->stream : nullptr; }

int osw_ingest_mean_square(int32_t device, const int16_t* pcm, int64_t n_frames, int32_t channels, float* out_mean) {
    return guard([&] {
        REQUIRE(pcm && out_mean, "null argument");
        REQUIRE(n_frames >= 1 && channels >= 1 && channels <= 64, "bad PCM shape");
        IngestDev& g = ingest_dev(device);
        std::lock_guard<std::mutex> lk(g.mu);
        DeviceScope dev_scope_((device));
        const size_t n = (size_t)n_frames * channels;
        grow(g.in, g.in_cap, n, g.owned);
        HIPCHK(hipMemcpyAsync(g.in, pcm, n * 2, hipMemcpyHostToDevice, g.s));
        *out_mean = ingest_mean_square(g, g.in, n_frames, channels);
    });
}

int osw_ingest_apply_gain(int32_t device, const int16_t* pcm, int64_t n_frames, int32_t channels, int32_t apply_gain,
                          float gain, int16_t* out) {
    return guard([&] {
        REQUIRE(pcm && out, "null argument");
        REQUIRE(n_frames >= 1 && channels >= 1 && channels <= 64, "bad PCM shape");
        IngestDev& g = ingest_dev(device);
        std::lock_guard<std::mutex> lk(g.mu);
        DeviceScope dev_scope_((device));
        const size_t n = (size_t)n_frames * channels;
        grow(g.in, g.in_cap, n, g.owned);
        grow(g.out, g.out_cap, (size_t)n_frames, g.owned);
        HIPCHK(hipMemcpyAsync(g.in, pcm, n * 2, hipMemcpyHostToDevice, g.s));
        launch_ingest_gain(g.in, n_frames, channels, apply_gain, gain, g.out, g.s);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(out, g.out, (size_t)n_frames * 2, hipMemcpyDeviceToHost, g.s));
        HIPCHK(hipStreamSynchronize(g.s));
    });
}

int osw_ingest_resample(int32_t device, const int16_t* pcm, int64_t n_in, int32_t up, int32_t down, const float* h,
                        int32_t n_h, int16_t* out, int64_t n_out) {
    return guard([&] {
        REQUIRE(pcm && h && out, "null argument");
        REQUIRE(n_in >= 2 && up >= 1 && down >= 1 && n_h >= 1 && (n_h & 1), "bad resample arguments");
        const int64_t want = (n_in * up) / down + ((n_in * up) % down ? 1 : 0);
        REQUIRE(n_out == want, "n_out must be ceil(n_in * up / down)");
        // resample_poly's zero padding of the filter (scipy/signal/_signaltools.py)
        const int64_t half_len = (n_h - 1) / 2;
        const int64_t pre = down - half_len % down;
        const int64_t pre_remove = (half_len + pre) / down;
        int64_t post = 0;
        while (upfirdn_output_len(n_h + pre + post, n_in, up, down) < n_out + pre_remove) ++post;
        const int64_t len_h = n_h + pre + post;
        const int64_t padlen = len_h + (up - len_h % up) % up;
        const int64_t hpp = padlen / up;
        // _pad_h: htf[p * hpp + j] = h_full[(hpp - 1 - j) * up + p]
        std::vector<float> full((size_t)padlen, 0.f), htf((size_t)padlen);
        for (int64_t i = 0; i < n_h; ++i) full[(size_t)(pre + i)] = h[i];
        for (int64_t p = 0; p < up; ++p)
            for (int64_t j = 0; j < hpp; ++j) htf[(size_t)(p * hpp + j)] = full[(size_t)((hpp - 1 - j) * up + p)];
        IngestDev& g = ingest_dev(device);
        std::lock_guard<std::mutex> lk(g.mu);
        DeviceScope dev_scope_((device));
        grow(g.in, g.in_cap, (size_t)n_in, g.owned);
        grow(g.out, g.out_cap, (size_t)n_out, g.owned);
        grow(g.taps, g.taps_cap, (size_t)padlen, g.owned);
        HIPCHK(hipMemcpyAsync(g.in, pcm, (size_t)n_in * 2, hipMemcpyHostToDevice, g.s));
        HIPCHK(hipMemcpyAsync(g.taps, htf.data(), htf.size() * 4, hipMemcpyHostToDevice, g.s));
        launch_ingest_resample(g.in, n_in, g.taps, (int)hpp, up, down, pre_remove, n_out, g.out, g.s);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(out, g.out, (size_t)n_out * 2, hipMemcpyDeviceToHost, g.s));
        HIPCHK(hipStreamSynchronize(g.s));
    });
}

}  // extern "C"
