// C-ABI host side of librescore (see include/rescore.h): weight packing, ragged
// sequence scheduling into launch chunks, and the per-chunk kernel pipeline.
//
// Scheduling replaces the reference's DataLoader of 32 padded rows
// (MLM_PLL/main.py:57-70, RescoreBert/main.py:71-79): all sequences of a call are
// flattened into ragged token rows and cut into chunks of <= max_rows rows, so every
// GEMM launch sees tens of thousands of rows and no padding tokens.
#include <map>
#include <string>
#include <vector>
#include <cstring>
#include <cstdio>
#include <cmath>
#include <algorithm>

#include "common.h"
#include "../../include/rescore.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPTRY(expr)                                                                   \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess)                                                          \
            return fail(RS_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
    } while (0)

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t n) {
        if (n <= bytes) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        hipError_t e = hipMalloc(&p, n);
        if (e == hipSuccess) bytes = n;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T> T* as() const { return (T*)p; }
};

struct Layer {
    f16 *wqkv, *wo, *w1, *w2;       // operand images of the precision mode (kx parts, planar)
    f16 *iqkv = nullptr, *io = nullptr, *i1 = nullptr, *i2 = nullptr;   // fp16x3: interleaved two-part
                                    // images [W_hi | W_lo*64] of the split-operand GEMMs (ldw = 2K)
    float *bqkv, *bo, *b1, *b2, *g1, *be1, *g2, *be2;
};

struct Chunk {
    int s0, s1, rows;
    int urows = 0;     // layer-0 unique rows (dedup mode), 0 = dedup off for this chunk
    int max_len = 0;   // longest sequence of the chunk (attention kernel choice)
};

}  // namespace

struct rs_model {
    rs_bert_cfg cfg{};
    int device = 0;
    bool finalized = false;
    std::map<std::string, std::vector<float>> host;   // fp32 state_dict staged until finalize
    std::vector<void*> allocs;                          // packed weights
    // packed weights
    float *word32 = nullptr, *pos32 = nullptr, *type32 = nullptr, *eg = nullptr, *eb = nullptr;
    std::vector<Layer> layers;
    f16* wt = nullptr;  float *bt = nullptr, *gt = nullptr, *bet = nullptr;   // MLM transform
    f16* wdec = nullptr; float* bdec = nullptr; int vpad = 0;                // tied decoder
    float *wlin = nullptr, *blin = nullptr;                                   // RescoreBert linear
    // workspace
    int64_t max_rows = 0;
    int s_cap = 0, r_pad = 0, m_pad = 0;
    int kx = 1;                 // fp16 operand image width (1: fp16, 3: fp16x3)
    bool x3s_w = false;         // the split-operand weight images exist (fp16x3, every projection
                                // weight |w| < 1023.75 so that 64 W_hi is finite in the x3s K loop)
    DevBuf xst, h16, t32, qkv, ctx, inter;   // xst: (mean, rstd) of the pre-LN rows in t32
    DevBuf xst1;                // statistics of the post-attention stream (deferred residual)
    DevBuf lnx, lncnt, lnerr;   // EPI_LNRES_IMG: per-tile row statistics, gang-ticket words (left
                                // zeroed by every launch), sticky statistics-wait timeout flag
    DevBuf ctxq, resq, tq32, hq32, hq16, interq, lab, llog, part, rowlp_tmp;
    DevBuf meta, hypoff;
    f16* emb_dst = nullptr;     // MODE_EMB output (rs_token_embed / rs_bertscore_recall)
    DevBuf emb, plan;           // rs_bertscore_recall: token embeddings, work-item plan
    DevBuf flag;                // non-finite-output flag of the last scoring call(s) (range guard)
    bool sync_check = true;     // scoring calls synchronise and report their flags (rs_model_set_sync_check)
    int* pinned_flag = nullptr;
    int* pinned_plan = nullptr;
    size_t pinned_plan_cap = 0;
    hipEvent_t plan_done = nullptr;
    std::vector<int> pinned_dummy;
    int* pinned = nullptr;
    size_t pinned_cap = 0;
    hipEvent_t upload_done = nullptr;
    // call ordering across streams: the end of the last call's work (any stream); a call on another
    // stream first makes its stream wait for it (CallOrder)
    hipEvent_t call_done = nullptr;
    hipStream_t last_stream = nullptr;
    bool have_last = false;
    bool order_lost = false;     // a call could not record call_done (order_begin reports it)
    // profiling
    bool prof = false;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    struct Rec { int kind; hipEvent_t a, b; double flops; };
    std::vector<Rec> recs;
    double prof_ms[RS_K_COUNT] = {};
    int64_t prof_n[RS_K_COUNT] = {};
    double prof_flops[RS_K_COUNT] = {};
};

namespace {

// Weight W [rows, cols] (nn.Linear [out, in]) -> fp16 operand image [rows_pad, kx*cols]:
// kx == 1: [hi]; kx == 3: [hi | lo*64 | hi/64] (pairs with the activation image
// [hi | hi/64 | lo*64], common.h put_split: the factors keep lo out of the fp16 subnormals).
f16* upload_f16(rs_model* m, const std::vector<float>& src, size_t rows_pad, size_t cols, int kx,
                hipError_t* err) {
    std::vector<f16> tmp(rows_pad * cols * kx, (f16)0.0f);
    const size_t rows = src.size() / cols;
    for (size_t r = 0; r < rows; ++r)
        for (size_t c = 0; c < cols; ++c) {
            const float v = src[r * cols + c];
            const f16 hi = (f16)v;
            f16* row = tmp.data() + r * cols * kx;
            row[c] = hi;
            if (kx == 3) {
                row[cols + c] = (f16)((v - (float)hi) * 64.f);
                row[2 * cols + c] = (f16)((float)hi * (1.f / 64.f));
            }
        }
    void* p = nullptr;
    *err = hipMalloc(&p, tmp.size() * sizeof(f16));
    if (*err != hipSuccess) return nullptr;
    m->allocs.push_back(p);
    *err = hipMemcpy(p, tmp.data(), tmp.size() * sizeof(f16), hipMemcpyHostToDevice);
    return (f16*)p;
}

// Weight W [rows, cols] -> the split-operand GEMM's interleaved two-part image [rows, 2 cols]
// (common.h, kx == 2): per 32-column K-step [hi 32 | lo*64 32], the same hi / lo*64 values as the
// planar three-part image's first two parts.
f16* upload_il(rs_model* m, const std::vector<float>& src, size_t cols, hipError_t* err) {
    const size_t rows = src.size() / cols;
    std::vector<f16> tmp(rows * cols * 2, (f16)0.0f);
    for (size_t r = 0; r < rows; ++r)
        for (size_t c = 0; c < cols; ++c) {
            const float v = src[r * cols + c];
            const f16 hi = (f16)v;
            f16* row = tmp.data() + r * cols * 2;
            row[il_hi((int)c)] = hi;
            row[il_hi((int)c) + 32] = (f16)((v - (float)hi) * 64.f);
        }
    void* p = nullptr;
    *err = hipMalloc(&p, tmp.size() * sizeof(f16));
    if (*err != hipSuccess) return nullptr;
    m->allocs.push_back(p);
    *err = hipMemcpy(p, tmp.data(), tmp.size() * sizeof(f16), hipMemcpyHostToDevice);
    return (f16*)p;
}

// The split-operand K loop forms 64 W_hi in fp16 (k_gemm.hip kstep16): finite only for
// |W_hi| <= 1023.5, i.e. |w| < 1023.75.  A model with a larger projection weight runs its fp16x3
// layers in the K-concatenated form instead (no 64x factor on W_hi), which holds |w| <= 65504.
bool x3s_range_ok(const std::vector<float>& v) {
    for (float x : v)
        if (!(std::fabs(x) < 1023.75f)) return false;
    return true;
}

float* upload_f32(rs_model* m, const std::vector<float>& src, size_t n_pad, hipError_t* err) {
    std::vector<float> tmp(std::max(n_pad, src.size()), 0.0f);
    std::memcpy(tmp.data(), src.data(), src.size() * sizeof(float));
    void* p = nullptr;
    *err = hipMalloc(&p, tmp.size() * sizeof(float));
    if (*err != hipSuccess) return nullptr;
    m->allocs.push_back(p);
    *err = hipMemcpy(p, tmp.data(), tmp.size() * sizeof(float), hipMemcpyHostToDevice);
    return (float*)p;
}

// The fp16 operand images (fp16 and fp16x3 modes) hold |x| <= 65504: a weight beyond it
// would become inf in its hi part (and NaN in lo), where the reference's fp32 forward stays
// finite.  Checked once at finalize.
bool fp16_range_ok(const std::vector<float>& v) {
    for (float x : v)
        if (!(std::fabs(x) <= 65504.f)) return false;
    return true;
}

// Activations are checked through their consequence: an operand that leaves the fp16 range
// becomes inf (hi) / NaN (lo) in its image, and inf / NaN then reaches every score that
// depends on it (LayerNorm, softmax and the log-softmax turn it into NaN; the fp32 reference
// stays finite there).  One pass over a call's outputs sets a flag, the call synchronises
// its stream and fails with RS_EUNSUP instead of returning non-finite scores.
template <class T>
__global__ void __launch_bounds__(256) nonfinite_kernel(const T* __restrict__ v, size_t n, int* __restrict__ flag) {
    int bad = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        bad |= !__builtin_isfinite((float)v[i]);
    if (bad) flag[0] = 1;          // plain vector store; every writer stores the same value
}

// Reads the flags (non-finite output, statistics-wait timeout) after synchronising the stream,
// clears them and turns them into the call's error.
int report_flags(rs_model* m, hipStream_t st, const char* what) {
    if (!m->pinned_flag) HIPTRY(hipHostMalloc((void**)&m->pinned_flag, 8, hipHostMallocDefault));
    m->pinned_flag[0] = 0;
    m->pinned_flag[1] = 0;
    if (m->flag.p) HIPTRY(hipMemcpyAsync(m->pinned_flag, m->flag.p, 4, hipMemcpyDeviceToHost, st));
    if (m->lnerr.p) HIPTRY(hipMemcpyAsync(m->pinned_flag + 1, m->lnerr.p, 4, hipMemcpyDeviceToHost, st));
    HIPTRY(hipStreamSynchronize(st));
    const int bad = m->pinned_flag[0], lnto = m->pinned_flag[1];
    if (bad && m->flag.p) HIPTRY(hipMemset(m->flag.p, 0, 4));
    if (lnto) {
        HIPTRY(hipMemset(m->lnerr.p, 0, 4));
        return fail(RS_EHIP, "a residual-LayerNorm GEMM timed out waiting for its row statistics "
                             "(set RS_LNFUSE=0 to use the separate LayerNorm pass)");
    }
    if (bad)
        return fail(RS_EUNSUP, std::string("non-finite ") + what +
                                   ": an activation left the fp16 range of the operand images (|x| > 65504); "
                                   "the fp32 reference stays finite here");
    return RS_OK;
}

// End of every scoring call: one pass over its outputs sets the non-finite flag.  Synchronous
// mode (default): the call waits for its stream and reports the flags.  Deferred mode
// (rs_model_set_sync_check(m, 0)): the pass is only enqueued, the flags accumulate on the device
// and rs_check reports them, so pipelined callers keep their stream asynchronous.
template <class T>
int check_finite(rs_model* m, hipStream_t st, const T* p, size_t n, const char* what) {
    if (!m->flag.p) {
        HIPTRY(m->flag.ensure(4));
        HIPTRY(hipMemset(m->flag.p, 0, 4));
    }
    if (n > 0) {
        const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 2048);
        hipLaunchKernelGGL(nonfinite_kernel<T>, dim3(blocks), dim3(256), 0, st, p, n, m->flag.as<int>());
        HIPTRY(hipGetLastError());
    }
    if (!m->sync_check) return RS_OK;
    return report_flags(m, st, what);
}

// Start of every scoring call in synchronous mode: a timeout flag left by an earlier call that
// failed before its report is dropped (each call reports only its own).
int begin_call(rs_model* m, hipStream_t st) {
    if (m->sync_check && m->lnerr.p) HIPTRY(hipMemsetAsync(m->lnerr.p, 0, 4, st));
    if (m->sync_check && m->flag.p) HIPTRY(hipMemsetAsync(m->flag.p, 0, 4, st));
    return RS_OK;
}

// Calls on one model handle are ordered, whatever streams they come on: the handle's workspace,
// LayerNorm gang tickets and flags are shared by every call, so a call on a different stream than the
// previous call first makes its stream wait (device-side, hipStreamWaitEvent) for the previous call's
// work, and every call records the end of its own work in call_done (created at finalize on the
// model's device).  Host threads must still not share a handle.  A failed wait fails the call
// (RS_EHIP); a failed record cannot change the return of the call it ends, so it is sticky: the next
// call on the handle fails with RS_EHIP instead of running unordered.
int order_begin(rs_model* m, hipStream_t st) {
    if (m->order_lost) {
        m->order_lost = false;
        return fail(RS_EHIP, "the previous call on this handle could not record its end (hipEventRecord "
                             "failed): cross-stream ordering was lost; synchronise the device and retry");
    }
    if (m->have_last && st != m->last_stream && m->call_done)
        HIPTRY(hipStreamWaitEvent(st, m->call_done, 0));
    return RS_OK;
}
struct CallOrder {
    rs_model* m;
    hipStream_t st;
    CallOrder(rs_model* m_, hipStream_t st_) : m(m_), st(st_) {}
    ~CallOrder() {
        if (!m->call_done) return;                // not finalized: no call ran kernels
        if (hipEventRecord(m->call_done, st) == hipSuccess) {
            m->last_stream = st;
            m->have_last = true;
        } else {
            m->order_lost = true;
        }
    }
};
#define CALL_ORDER(m_, st_)                                   \
    if (int r_ = order_begin((m_), (st_))) return r_;         \
    CallOrder order_((m_), (st_))

int reserve_impl(rs_model* m, int64_t max_rows) {
    const rs_bert_cfg& c = m->cfg;
    if (max_rows < 512) return fail(RS_EARG, "max_rows must be >= 512");
    if (max_rows > (int64_t)1 << 26) return fail(RS_EARG, "max_rows too large");
    const int al = gemm_row_align();
    m->max_rows = max_rows;
    m->m_pad = (int)((max_rows + al - 1) / al * al);
    m->s_cap = (int)(max_rows / 3) + 1;
    m->r_pad = (m->s_cap + al - 1) / al * al;
    const size_t M = m->m_pad, R = m->r_pad, H = c.hidden, F = c.intermediate;
    HIPTRY(hipSetDevice(m->device));
    const size_t kx = m->kx;
    HIPTRY(m->xst.ensure(M * sizeof(float2)));
    HIPTRY(m->xst1.ensure(M * sizeof(float2)));
    HIPTRY(m->lnx.ensure(lnres_granules((int)M) * 8));
    HIPTRY(hipMemset(m->lnx.p, 0, m->lnx.bytes));               // granule tags start at 0 (never a launch's)
    if (!m->lncnt.p) {
        HIPTRY(m->lncnt.ensure(lnres_counter_bytes()));
        HIPTRY(hipMemset(m->lncnt.p, 0, m->lncnt.bytes));
    }
    HIPTRY(m->lnerr.ensure(16));
    HIPTRY(hipMemset(m->lnerr.p, 0, 16));
    HIPTRY(m->h16.ensure(M * H * 2 * kx));
    HIPTRY(m->t32.ensure(M * H * 4));
    HIPTRY(m->qkv.ensure(M * 3 * H * (kx == 3 ? 4 : 2)));
    HIPTRY(m->ctx.ensure(M * H * 2 * kx));
    HIPTRY(m->inter.ensure(M * F * 2 * kx));
    HIPTRY(m->ctxq.ensure(R * H * 2 * kx));
    HIPTRY(m->resq.ensure(R * H * 4));
    HIPTRY(m->tq32.ensure(R * H * 4));
    HIPTRY(m->hq32.ensure(R * H * 4));
    HIPTRY(m->hq16.ensure(R * H * 2 * kx));
    HIPTRY(m->interq.ensure(R * F * 2 * kx));
    HIPTRY(m->lab.ensure(R * 4));
    HIPTRY(m->llog.ensure(R * 4));
    if (c.heads_mask & RS_HEAD_MLM) HIPTRY(m->part.ensure(R * (size_t)(m->vpad / 64) * sizeof(float2)));
    // zero the padded activations once: GEMMs read pad rows (never stored back)
    HIPTRY(hipMemset(m->h16.p, 0, m->h16.bytes));
    HIPTRY(hipMemset(m->ctx.p, 0, m->ctx.bytes));
    HIPTRY(hipMemset(m->inter.p, 0, m->inter.bytes));
    HIPTRY(hipMemset(m->ctxq.p, 0, m->ctxq.bytes));
    HIPTRY(hipMemset(m->hq16.p, 0, m->hq16.bytes));
    HIPTRY(hipMemset(m->interq.p, 0, m->interq.bytes));
    HIPTRY(hipMemset(m->t32.p, 0, m->t32.bytes));    // pad rows of the residual stream stay finite
    HIPTRY(hipMemset(m->xst.p, 0, m->xst.bytes));
    HIPTRY(hipMemset(m->xst1.p, 0, m->xst1.bytes));
    return RS_OK;
}

const std::vector<float>* need(rs_model* m, const std::string& k, size_t n, std::string* missing) {
    auto it = m->host.find(k);
    if (it == m->host.end()) {
        if (missing->empty()) *missing = k + " (missing)";
        return nullptr;
    }
    if (it->second.size() != n) {
        if (missing->empty()) *missing = k + " (wrong size)";
        return nullptr;
    }
    return &it->second;
}

// ---- profiling helpers ----------------------------------------------------------------
hipEvent_t next_event(rs_model* m) {
    if (m->ev_used == m->ev_pool.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        m->ev_pool.push_back(e);
    }
    return m->ev_pool[m->ev_used++];
}

struct ProfScope {
    rs_model* m;
    hipStream_t st;
    int kind;
    double flops;
    hipEvent_t a = nullptr;
    ProfScope(rs_model* m_, hipStream_t st_, int kind_, double flops_) : m(m_), st(st_), kind(kind_), flops(flops_) {
        if (m->prof) {
            a = next_event(m);
            if (a) (void)hipEventRecord(a, st);
        }
    }
    ~ProfScope() {
        if (m->prof && a) {
            hipEvent_t b = next_event(m);
            if (b) {
                (void)hipEventRecord(b, st);
                m->recs.push_back({kind, a, b, flops});
            }
        }
    }
};

int gemm(rs_model* m, hipStream_t st, int kind, int epi, const f16* A, const f16* W, int m_valid,
         int N_pad, int K, EpiArgs ep, int n_flop_cols) {
    const int al = gemm_row_align();
    const int M_pad = (m_valid + al - 1) / al * al;
    ep.m_valid = m_valid;
    ProfScope ps(m, st, kind, 2.0 * m_valid * (double)n_flop_cols * K);
    HIPTRY(launch_gemm(epi, A, W, M_pad, N_pad, K, ep, st, kind == RS_K_OPROJ ? 1 : kind == RS_K_FFN2 ? 2 : 0));
    return RS_OK;
}

enum Mode { MODE_MLM = 0, MODE_CLS = 1, MODE_EMB = 2 };

// RS_OPROJ: "f16" (default in the fp16 precision mode: fp16-output O projection + fused
// residual/LayerNorm rows kernel) or "resln" (residual rebuilt in the GEMM's accumulators)
// (read per call, like RS_DEDUP, so a test can flip it in-process)
bool oproj_f16() {
    const char* e = getenv("RS_OPROJ");
    return !(e && !strcmp(e, "resln"));
}
// RS_LNRES_DEFER (fp16 mode, O-projection split): ln_res_rows writes only the statistics and
// the fp16 image of the post-attention stream x = LN0(x32) + o1 (o1 = fp16 O-projection
// output), so x never round-trips through HBM in fp32, and x is rebuilt downstream:
//   2 (default): BertOutput is a lean fp16-output GEMM (o2) and one second ln_res_rows pass
//                forms LN2(LN1(LN0(x32) + o1) + o2) — no residual traffic in any GEMM epilogue;
//   1: the BertOutput GEMM rebuilds x in its accumulator init (EpiArgs.res_o16) — slower: the
//      extra loads sit in front of the tile's first MFMA;
//   0: ln_res_rows writes x back into x32 and BertOutput reads it (EPI_RESLN_F32).
int lnres_defer() {
    const char* e = getenv("RS_LNRES_DEFER");
    return e ? atoi(e) : 2;
}
// RS_FFN2: "resln" (default) or "f16" (the O-projection split applied to BertOutput)
bool ffn2_f16() {
    const char* e = getenv("RS_FFN2");
    return e && !strcmp(e, "f16");
}

// RS_X3S (fp16x3 mode, default 1): the encoder projections run as split-operand GEMMs
// (gemm_x3s_kernel: two-part activation images, three fp16 products formed in registers, fp32
// outputs + ln_res32 rows for the residual blocks); 0 = the K-concatenated three-part form.
// Read per call (tests flip it in-process).
bool x3s_on(const rs_model* m) {
    const char* e = getenv("RS_X3S");
    return !(e && !strcmp(e, "0")) && m->x3s_w && m->cfg.hidden % 256 == 0 && m->cfg.intermediate % 256 == 0;
}
// RS_X3S_IMGRES (split-operand layers, default 1): the residual stream is held only as the
// two-part image of the normalised hidden state (ln_res_img: 12 B per element per residual
// block, no fp32 pre-LN stream or statistics); 0 = ln_res32 over the fp32 pre-LN stream.
bool x3s_imgres_on() {
    const char* e = getenv("RS_X3S_IMGRES");
    return !(e && !strcmp(e, "0"));
}
// RS_LNFUSE (image-held residual; default 1): the residual add + LayerNorm of both blocks run in
// the O-projection / BertOutput GEMM epilogues (EPI_LNRES_IMG: full rows through an in-launch
// exchange of row statistics) instead of as ln_res_img passes (RS_LNFUSE=0).  Read per call.
bool lnfuse_on(const rs_bert_cfg& cf) {
    const char* e = getenv("RS_LNFUSE");
    return !(e && !strcmp(e, "0")) && cf.hidden % 256 == 0 && cf.hidden <= 1024;
}

// Runs the encoder + head over sequences [c.s0, c.s1) (one chunk).
int run_chunk(rs_model* m, hipStream_t st, const int* d_tok, const SeqMeta& sm, const Chunk& c,
              int mode, float* d_out_rows /* indexed by sequence */) {
    const rs_bert_cfg& cf = m->cfg;
    const int H = cf.hidden, F = cf.intermediate, nh = cf.heads, kx = m->kx;
    const bool q32 = kx == 3;                 // fp16x3: QKV kept in fp32 for attention
    const int qkv_epi = q32 ? EPI_BIAS_F32 : EPI_BIAS_F16;
    const int rows = c.rows, ns = c.s1 - c.s0;
    const bool dedup = c.urows > 0;           // layer-0 Q/K/V over unique rows (MLM; fp16, or fp16x3 split)
    const bool x3s = kx == 3 && x3s_on(m);    // split-operand GEMMs: full-row images are two-part
    const int kxf = x3s ? 2 : kx;             // width factor of the full-row operand images
    const bool imgres = x3s && x3s_imgres_on();  // residual stream = the two-part image in h16
    const bool lnfuse = imgres && lnfuse_on(cf);  // ... closed in the residual GEMMs' epilogues
    float2* xst = m->xst.as<float2>();
    f16* h16 = m->h16.as<f16>();
    float* t32 = m->t32.as<float>();     // residual stream, pre-LN fp32 (LN rebuilt from xst)
    void* qkv = m->qkv.p;
    f16* ctx = m->ctx.as<f16>();
    f16* inter = m->inter.as<f16>();
    {
        ProfScope ps(m, st, RS_K_OTHER, 0);
        // dedup: the per-copy pass keeps only the fp32 residual + LN statistics; the layer-0
        // GEMM operand is built over the chunk's unique rows (plan_unique_rows)
        // (split-operand dedup: every copy row's image stays in h16 — it is the layer-0
        // residual — and the unique rows' image goes to the idle FFN buffer)
        HIPTRY(launch_embed_ln(d_tok, sm, c.s0, c.s1, 0, cf.mask_id, cf.vocab, m->word32, m->pos32,
                               m->type32, m->eg, m->eb, cf.ln_eps, H, imgres ? nullptr : t32, imgres ? nullptr : xst,
                               dedup && !x3s ? nullptr : h16, kxf, st));
        if (dedup)
            HIPTRY(launch_embed_unique(d_tok, sm, c.s0, c.s1, cf.mask_id, cf.vocab, m->word32, m->pos32,
                                       m->type32, m->eg, m->eb, cf.ln_eps, H, x3s ? inter : h16, kxf, st));
    }
    EpiArgs ep{};
    // split-operand GEMM over m_valid rows: A two-part image, W rows of ldw halfs; profiled as
    // MFMA work (three products of logical K)
    auto gx = [&](int kind, int epi, const f16* A, const f16* W, int ldw, int m_valid, int N, int K, EpiArgs e,
                  int n_flop_cols) -> int {
        const int al = gemm_row_align();
        e.m_valid = m_valid;
        ProfScope ps(m, st, kind, 2.0 * m_valid * (double)n_flop_cols * 3.0 * K);
        const int M_pad = (m_valid + al - 1) / al * al;
        HIPTRY(launch_gemm_x3s(epi, A, W, ldw, M_pad, N, K, e, st));
        return RS_OK;
    };
    auto gelu_ep = [&](const float* bias, f16* out) {
        EpiArgs e{};
        e.bias = bias; e.out = out; e.ldc = kx * F; e.kx = kx; e.nlog = F;
        return e;
    };
    // residual GEMM: t32 <- acc + bias + LN(t32) (in place: a tile reads and writes only its own
    // rows x columns), LN given by the statistics in xst and the LN parameters (lg, lb)
    auto resln_ep = [&](const float* bias, const float* lg, const float* lb) {
        EpiArgs e{};
        e.bias = bias; e.res = t32; e.res_stats = xst; e.res_g = lg; e.res_b = lb; e.out = t32; e.ldc = H;
        return e;
    };
    for (int li = 0; li < cf.layers; ++li) {
        const Layer& L = m->layers[li];
        const bool last = mode != MODE_EMB && li == cf.layers - 1;   // query-row-only layer
        // LayerNorm that produced this layer's input (embeddings LN, or the previous BertOutput LN)
        const float* pg = li ? m->layers[li - 1].g2 : m->eg;
        const float* pb = li ? m->layers[li - 1].be2 : m->eb;
        ep = EpiArgs{};
        ep.bias = L.bqkv; ep.out = qkv; ep.ldc = 3 * H;
        const bool uq = dedup && li == 0;
        const void* qdense = nullptr;
        const char* lq_env = getenv("RS_LASTQ");      // "0": full Q/K/V GEMM at the last layer
        if (last && !uq && !(lq_env && !strcmp(lq_env, "0"))) {
            // Query-row-only layer: K and V for every row (rows H..3H of the fused weight,
            // written into columns H..3H of qkv), Q only for the scored row of each sequence
            // (gathered operand rows -> dense [sequence, H] in the idle tq32 buffer)
            const size_t esz = q32 ? 4 : 2;
            ep.bias = L.bqkv + H;
            ep.out = (char*)qkv + H * esz;
            if (x3s) {
                if (int r = gx(RS_K_QKV, EPI_BIAS_F32, h16, L.iqkv + (size_t)H * 2 * H, 2 * H, rows, 2 * H, H, ep, 2 * H))
                    return r;
            } else if (int r = gemm(m, st, RS_K_QKV, qkv_epi, h16, L.wqkv + (size_t)H * kx * H, rows, 2 * H, kx * H, ep,
                                    2 * H)) return r;
            f16* hq16g = m->hq16.as<f16>();
            {
                ProfScope ps(m, st, RS_K_OTHER, 0);
                HIPTRY(launch_gather_query_rows(h16, kxf * H, sm, c.s0, c.s1, 0, hq16g, st));
            }
            EpiArgs eq{};
            eq.bias = L.bqkv; eq.out = m->tq32.p; eq.ldc = H;
            if (x3s) {
                if (int r = gx(RS_K_QKV, EPI_BIAS_F32, hq16g, L.iqkv, 2 * H, ns, H, H, eq, H)) return r;
            } else if (int r = gemm(m, st, RS_K_QKV, qkv_epi, hq16g, L.wqkv, ns, H, kx * H, eq, H)) return r;
            qdense = m->tq32.p;
        } else if (x3s) {
            if (int r = gx(RS_K_QKV, EPI_BIAS_F32, uq ? inter : h16, L.iqkv, 2 * H, uq ? c.urows : rows, 3 * H, H, ep,
                           last ? 2 * H : 3 * H)) return r;
        } else if (int r = gemm(m, st, RS_K_QKV, qkv_epi, h16, L.wqkv, uq ? c.urows : rows, 3 * H, kx * H, ep,
                                last ? 2 * H : 3 * H)) return r;
        if (!last && x3s) {
            // fp16x3 split-operand layer: projections write fp32 (o32 in the dead QKV buffer),
            // the residual blocks close in ln_res32 (x32 <- LN(x32) + o32, next two-part image)
            {
                ProfScope ps(m, st, RS_K_ATTN, 0);
                HIPTRY(launch_attention_full(qkv, true, sm, c.s0, c.s1, 0, H, nh, ctx, 2, st, uq, c.max_len));
            }
            float* o32 = (float*)qkv;
            // residual block: h16 <- image(LN(A·Wᵀ + b + h16)) in the GEMM epilogue (lnfuse), or
            // an fp32 GEMM output closed by a separate residual + LayerNorm pass
            auto lnres_ep = [&](const float* bias, const float* g, const float* be) {
                EpiArgs e{};
                e.bias = bias; e.out = h16; e.ldc = 2 * H; e.nlog = H; e.res_g = g; e.res_b = be;
                e.ln_eps = cf.ln_eps; e.lnx = m->lnx.p; e.lncnt = m->lncnt.as<unsigned>();
                e.lnerr = m->lnerr.as<unsigned>();
                // RS_LNFUSE_DIAG=8 (tests; read per call): every statistics / gang wait times out at
                // once (the RS_EHIP path); no other bit is honoured (no diagnostic changes scores)
                e.diag = (getenv("RS_LNFUSE_DIAG") ? atoi(getenv("RS_LNFUSE_DIAG")) : 0) & 8;
                return e;
            };
            if (lnfuse) {
                if (int r = gx(RS_K_OPROJ, EPI_LNRES_IMG, ctx, L.io, 2 * H, rows, H, H, lnres_ep(L.bo, L.g1, L.be1), H))
                    return r;
            } else {
                ep = EpiArgs{}; ep.bias = L.bo; ep.out = o32; ep.ldc = H;
                if (int r = gx(RS_K_OPROJ, EPI_BIAS_F32, ctx, L.io, 2 * H, rows, H, H, ep, H)) return r;
                ProfScope ps(m, st, RS_K_OTHER, 0);
                if (imgres) HIPTRY(launch_ln_res_img(h16, o32, rows, L.g1, L.be1, cf.ln_eps, H, st));
                else HIPTRY(launch_ln_res32(t32, xst, xst, pg, pb, o32, rows, L.g1, L.be1, cf.ln_eps, H, h16, 2, st));
            }
            ep = EpiArgs{}; ep.bias = L.b1; ep.out = inter; ep.ldc = 2 * F; ep.kx = 2; ep.nlog = F;
            if (int r = gx(RS_K_FFN1, EPI_GELU_F16, h16, L.i1, 2 * H, rows, F, H, ep, F)) return r;
            if (lnfuse) {
                if (int r = gx(RS_K_FFN2, EPI_LNRES_IMG, inter, L.i2, 2 * F, rows, H, F, lnres_ep(L.b2, L.g2, L.be2), H))
                    return r;
            } else {
                ep = EpiArgs{}; ep.bias = L.b2; ep.out = o32; ep.ldc = H;
                if (int r = gx(RS_K_FFN2, EPI_BIAS_F32, inter, L.i2, 2 * F, rows, H, F, ep, H)) return r;
                ProfScope ps(m, st, RS_K_OTHER, 0);
                if (imgres) HIPTRY(launch_ln_res_img(h16, o32, rows, L.g2, L.be2, cf.ln_eps, H, st));
                else HIPTRY(launch_ln_res32(t32, xst, xst, L.g1, L.be1, o32, rows, L.g2, L.be2, cf.ln_eps, H, h16, 2, st));
            }
        } else if (!last) {
            {
                ProfScope ps(m, st, RS_K_ATTN, 0);
                HIPTRY(launch_attention_full(qkv, q32, sm, c.s0, c.s1, 0, H, nh, ctx, kx, st, uq, c.max_len));
            }
            const bool fp16_split = kx == 1 && oproj_f16();
            const int dmode = fp16_split && !ffn2_f16() ? lnres_defer() : 0;
            const bool defer = dmode != 0;
            // O-projection output (fp16): the dead QKV buffer when the BertOutput GEMM reads it
            // back (deferred residual: it must survive FFN1), else the (free) FFN1 buffer
            f16* o16 = defer ? (f16*)qkv : inter;
            if (fp16_split) {
                // O projection as a persistent fp16-output GEMM; the residual add + LayerNorm
                // move into ln_res_rows, off the GEMM's critical path
                ep = EpiArgs{}; ep.bias = L.bo; ep.out = o16; ep.ldc = H;
                if (int r = gemm(m, st, RS_K_OPROJ, EPI_BIAS_F16, ctx, L.wo, rows, H, H, ep, H)) return r;
                ProfScope ps(m, st, RS_K_OTHER, 0);
                HIPTRY(launch_ln_res_rows(t32, xst, defer ? m->xst1.as<float2>() : xst, pg, pb, o16, rows, L.g1, L.be1,
                                          cf.ln_eps, H, h16, !defer, st));
            } else {
                ep = resln_ep(L.bo, pg, pb);
                if (int r = gemm(m, st, RS_K_OPROJ, EPI_RESLN_F32, ctx, L.wo, rows, H, kx * H, ep, H)) return r;
                ProfScope ps(m, st, RS_K_OTHER, 0);
                HIPTRY(launch_ln_rows(t32, rows, L.g1, L.be1, cf.ln_eps, H, nullptr, xst, h16, kx, st));
            }
            ep = gelu_ep(L.b1, inter);
            if (int r = gemm(m, st, RS_K_FFN1, EPI_GELU_F16, h16, L.w1, rows, F, kx * H, ep, F)) return r;
            if (dmode == 2) {
                // BertOutput as a persistent fp16-output GEMM into the (free) ctx buffer; both
                // residual blocks of the layer are closed by one ln_res_rows pass
                ep = EpiArgs{}; ep.bias = L.b2; ep.out = ctx; ep.ldc = H;
                if (int r = gemm(m, st, RS_K_FFN2, EPI_BIAS_F16, inter, L.w2, rows, H, F, ep, H)) return r;
                ProfScope ps(m, st, RS_K_OTHER, 0);
                HIPTRY(launch_ln_res_rows(t32, xst, xst, pg, pb, o16, rows, L.g2, L.be2, cf.ln_eps, H, h16, true, st,
                                          m->xst1.as<float2>(), L.g1, L.be1, ctx));
            } else if (kx == 1 && ffn2_f16()) {
                // same split for BertOutput: fp16-output GEMM into the (free) ctx buffer
                ep = EpiArgs{}; ep.bias = L.b2; ep.out = ctx; ep.ldc = H;
                if (int r = gemm(m, st, RS_K_FFN2, EPI_BIAS_F16, inter, L.w2, rows, H, F, ep, H)) return r;
                ProfScope ps(m, st, RS_K_OTHER, 0);
                HIPTRY(launch_ln_res_rows(t32, xst, xst, L.g1, L.be1, ctx, rows, L.g2, L.be2, cf.ln_eps, H, h16, true, st));
            } else {
                ep = resln_ep(L.b2, L.g1, L.be1);
                if (defer) {
                    ep.res_stats = m->xst1.as<float2>();
                    ep.res_o16 = o16; ep.res_stats0 = xst; ep.res_g0 = pg; ep.res_b0 = pb;
                }
                if (int r = gemm(m, st, RS_K_FFN2, EPI_RESLN_F32, inter, L.w2, rows, H, kx * F, ep, H)) return r;
                ProfScope ps(m, st, RS_K_OTHER, 0);
                HIPTRY(launch_ln_rows(t32, rows, L.g2, L.be2, cf.ln_eps, H, nullptr, xst, h16, kx, st));
            }
        } else {
            // last layer: only the scored row of every sequence (one row per sequence)
            f16* ctxq = m->ctxq.as<f16>();
            float* resq = m->resq.as<float>();
            float* tq = m->tq32.as<float>();
            float* hq32 = m->hq32.as<float>();
            f16* hq16 = m->hq16.as<f16>();
            f16* interq = m->interq.as<f16>();
            {
                ProfScope ps(m, st, RS_K_ATTN, 0);
                HIPTRY(launch_attention_query(qkv, q32, t32, xst, pg, pb, sm, c.s0, c.s1, 0, H, nh, ctxq, resq, kx, st,
                                              qdense, imgres ? h16 : nullptr));
            }
            ep = EpiArgs{}; ep.bias = L.bo; ep.res = resq; ep.out = tq; ep.ldc = H;
            if (int r = gemm(m, st, RS_K_OPROJ, EPI_RES_F32, ctxq, L.wo, ns, H, kx * H, ep, H)) return r;
            { ProfScope ps(m, st, RS_K_OTHER, 0); HIPTRY(launch_ln_rows(tq, ns, L.g1, L.be1, cf.ln_eps, H, hq32, nullptr, hq16, kx, st)); }
            ep = gelu_ep(L.b1, interq);
            if (int r = gemm(m, st, RS_K_FFN1, EPI_GELU_F16, hq16, L.w1, ns, F, kx * H, ep, F)) return r;
            ep = EpiArgs{}; ep.bias = L.b2; ep.res = hq32; ep.out = tq; ep.ldc = H;
            if (int r = gemm(m, st, RS_K_FFN2, EPI_RES_F32, interq, L.w2, ns, H, kx * F, ep, H)) return r;
            { ProfScope ps(m, st, RS_K_OTHER, 0); HIPTRY(launch_ln_rows(tq, ns, L.g2, L.be2, cf.ln_eps, H, hq32, nullptr, hq16, kx, st)); }
        }
    }
    if (mode == MODE_EMB) {
        const Layer& L = m->layers[cf.layers - 1];
        ProfScope ps(m, st, RS_K_OTHER, 0);
        HIPTRY(launch_embed_out(t32, xst, L.g2, L.be2, sm, c.s0, c.s1, 0, H, m->emb_dst, st, imgres ? h16 : nullptr,
                                m->kx == 3));
        return RS_OK;
    }
    float* hq32 = m->hq32.as<float>();
    f16* hq16 = m->hq16.as<f16>();
    float* tq = m->tq32.as<float>();
    if (mode == MODE_MLM) {
        ep = EpiArgs{}; ep.bias = m->bt; ep.out = tq; ep.ldc = H;
        if (int r = gemm(m, st, RS_K_DECODER, EPI_GELU_F32, hq16, m->wt, ns, H, kx * H, ep, H)) return r;
        { ProfScope ps(m, st, RS_K_OTHER, 0); HIPTRY(launch_ln_rows(tq, ns, m->gt, m->bet, cf.ln_eps, H, hq32, nullptr, hq16, kx, st)); }
        int* lab = m->lab.as<int>();
        float* ll = m->llog.as<float>();
        { ProfScope ps(m, st, RS_K_OTHER, 0); HIPTRY(launch_gather_labels(d_tok, sm, c.s0, c.s1, lab, st)); }
        ep = EpiArgs{}; ep.bias = m->bdec; ep.n_valid = cf.vocab; ep.lse_part = m->part.as<float2>();
        ep.n_parts = m->vpad / 64; ep.label = lab; ep.label_logit = ll;
        if (int r = gemm(m, st, RS_K_DECODER, EPI_LSE, hq16, m->wdec, ns, m->vpad, kx * H, ep, cf.vocab)) return r;
        ProfScope ps(m, st, RS_K_OTHER, 0);
        HIPTRY(launch_lse_finalize(m->part.as<float2>(), m->vpad / 64, ll, ns, d_out_rows + c.s0, st));
    } else {
        ProfScope ps(m, st, RS_K_OTHER, 0);
        HIPTRY(launch_cls_linear(hq32, ns, H, m->wlin, m->blin, d_out_rows + c.s0, st));
    }
    return RS_OK;
}

// Host-side sequence list (structure of arrays) for one call.
struct SeqList {
    std::vector<int> tok_off, len, mask, query, label, row, urow_h, urow_m;
    void push(int to, int T, int mp, int q, int lb) {
        tok_off.push_back(to); len.push_back(T); mask.push_back(mp); query.push_back(q);
        label.push_back(lb); row.push_back(0); urow_h.push_back(0); urow_m.push_back(0);
    }
    size_t size() const { return len.size(); }
};

// Layer-0 dedup (MLM_PLL): the masked copies of one hypothesis share every layer-0 input row
// except the masked one, so the layer-0 QKV projection runs over UNIQUE rows: per hypothesis
// (within a chunk) its T original rows, then one [MASK] row per copy.  urow_h[s] = first
// unique row of the hypothesis, urow_m[s] = the copy's masked row (chunk-local).  Returns the
// chunk's unique-row count, or 0 when a sequence has no mask position (dedup not applicable).
int plan_unique_rows(SeqList& sl, int s0, int s1) {
    int u = 0, base = 0;
    for (int s = s0; s < s1; ++s) {
        if (sl.mask[s] < 0) return 0;
        if (s == s0 || sl.tok_off[s] != sl.tok_off[s - 1] || sl.len[s] != sl.len[s - 1]) {
            base = u;
            u += sl.len[s];
        }
        sl.urow_h[s] = base;
        sl.urow_m[s] = u++;
    }
    return u;
}

// Chunks the sequence list, uploads metadata, runs every chunk.  out_rows: one float per
// sequence.  Extra int arrays (e.g. hypothesis -> sequence offsets) ride in the same upload.
int run_all(rs_model* m, hipStream_t st, const int* d_tok, SeqList& sl, int mode, float* out_rows,
            const std::vector<int>* extra, int** d_extra, const int* d_label = nullptr) {
    if (!m->finalized) return fail(RS_ESTATE, "rs_model_finalize not called");
    if (mode == MODE_MLM && !(m->cfg.heads_mask & RS_HEAD_MLM)) return fail(RS_ESTATE, "model has no MLM head");
    if (mode == MODE_CLS && !(m->cfg.heads_mask & RS_HEAD_CLS)) return fail(RS_ESTATE, "model has no CLS linear head");
    if (m->max_rows == 0)
        if (int r = reserve_impl(m, 65536)) return r;
    HIPTRY(hipSetDevice(m->device));
    if (int r = begin_call(m, st)) return r;
    const size_t S = sl.size();
    std::vector<Chunk> chunks;
    // Chunk rows: with the fused residual + LayerNorm GEMMs (lnfuse), a chunk of P row panels runs
    // ceil(P / G) rounds of whole panels on G = gemm_lnres_workgroups / (H / 256) gangs, so the
    // chunks are cut at a multiple of 256 * G rows (bert-base on 256 CUs: 85 gangs, 21760 rows;
    // 262144 -> 261120 rows = 12 full rounds instead of 12 + a 4-panel 13th).  RS_CHUNK_ALIGN=0
    // keeps max_rows (read per call).
    int64_t cap = m->max_rows;
    {
        const char* ca = getenv("RS_CHUNK_ALIGN");
        const bool lnf = m->kx == 3 && x3s_on(m) && x3s_imgres_on() && lnfuse_on(m->cfg);
        const int ntn = m->cfg.hidden / 256;
        if (lnf && !(ca && !strcmp(ca, "0")) && ntn > 0) {
            const int64_t unit = (int64_t)256 * (gemm_lnres_workgroups(m->cfg.hidden) / ntn);
            if (unit > 0 && cap >= unit) cap = cap / unit * unit;
        }
    }
    int rows = 0, s0 = 0, max_len = 0;
    for (size_t s = 0; s < S; ++s) {
        const int T = sl.len[s];
        if (T > m->cfg.max_pos) return fail(RS_EUNSUP, "sequence longer than max_position_embeddings");
        if (T < 1) return fail(RS_EARG, "empty sequence");
        if (T > m->max_rows) return fail(RS_EARG, "sequence longer than the reserved rows");
        if (rows + T > cap || (int)s - s0 >= m->s_cap) {
            chunks.push_back({s0, (int)s, rows, 0, max_len});
            s0 = (int)s;
            rows = 0;
            max_len = 0;
        }
        sl.row[s] = rows;
        rows += T;
        max_len = std::max(max_len, T);
    }
    if (S) chunks.push_back({s0, (int)S, rows, 0, max_len});
    // layer-0 dedup: MLM mode, fp16 operands, >= 2 layers (layer 0 is not the query-only layer)
    const char* dedup_s = getenv("RS_DEDUP");      // read per call (tests flip it)
    const int dedup_env = dedup_s ? atoi(dedup_s) : 1;
    // fp16x3: the split-operand layer with the image-held residual (its attention kernel reads
    // the unique rows for chunks with T <= 64)
    const bool x3_dedup = m->kx == 3 && x3s_on(m) && x3s_imgres_on();
    if (dedup_env && mode == MODE_MLM && (m->kx == 1 || x3_dedup) && m->cfg.layers >= 2)
        for (Chunk& c : chunks)
            if (m->kx == 1 || c.max_len <= 64) c.urows = plan_unique_rows(sl, c.s0, c.s1);

    // one upload of all metadata through a pinned staging buffer
    const size_t n_extra = extra ? extra->size() : 0;
    const size_t n_int = 8 * S + n_extra;
    if (m->upload_done) HIPTRY(hipEventSynchronize(m->upload_done));
    if (n_int > m->pinned_cap) {
        if (m->pinned) (void)hipHostFree(m->pinned);
        m->pinned = nullptr;
        m->pinned_cap = 0;
        HIPTRY(hipHostMalloc((void**)&m->pinned, std::max<size_t>(n_int, 1) * 4, hipHostMallocDefault));
        m->pinned_cap = n_int;
    }
    int* p = m->pinned;
    const std::vector<int>* cols[8] = {&sl.tok_off, &sl.len, &sl.mask, &sl.query, &sl.label, &sl.row,
                                       &sl.urow_h, &sl.urow_m};
    for (int k = 0; k < 8; ++k) std::memcpy(p + k * S, cols[k]->data(), S * 4);
    if (n_extra) std::memcpy(p + 8 * S, extra->data(), n_extra * 4);
    HIPTRY(m->meta.ensure(std::max<size_t>(n_int, 1) * 4));
    HIPTRY(hipMemcpyAsync(m->meta.p, p, n_int * 4, hipMemcpyHostToDevice, st));
    if (!m->upload_done) HIPTRY(hipEventCreateWithFlags(&m->upload_done, hipEventDisableTiming));
    HIPTRY(hipEventRecord(m->upload_done, st));
    int* d = m->meta.as<int>();
    if (d_label) HIPTRY(hipMemcpyAsync(d + 4 * S, d_label, S * 4, hipMemcpyDeviceToDevice, st));
    SeqMeta sm{d, d + S, d + 2 * S, d + 3 * S, d + 4 * S, d + 5 * S, d + 6 * S, d + 7 * S};
    if (d_extra) *d_extra = d + 8 * S;
    for (const Chunk& c : chunks)
        if (int r = run_chunk(m, st, d_tok, sm, c, mode, out_rows)) return r;
    return RS_OK;
}

void prof_collect(rs_model* m) {
    if (m->recs.empty()) return;
    (void)hipEventSynchronize(m->recs.back().b);
    for (auto& r : m->recs) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
            m->prof_ms[r.kind] += ms;
            m->prof_n[r.kind] += 1;
            m->prof_flops[r.kind] += r.flops;
        }
    }
    m->recs.clear();
    m->ev_used = 0;
}

}  // namespace

// =======================================================================================
extern "C" {

int rs_version(void) { return 1; }

const char* rs_last_error(void) { return g_err.c_str(); }

int rs_model_create(const rs_bert_cfg* cfg, int device, rs_model** out) {
    if (!cfg || !out) return fail(RS_EARG, "null argument");
    const rs_bert_cfg& c = *cfg;
    if (c.hidden <= 0 || c.hidden % 256 || c.hidden > 1024) return fail(RS_EUNSUP, "hidden must be 256/512/768/1024");
    if (c.heads <= 0 || c.hidden / c.heads != 64 || c.hidden % c.heads) return fail(RS_EUNSUP, "head_dim must be 64");
    if (c.intermediate <= 0 || c.intermediate % 128) return fail(RS_EUNSUP, "intermediate must be a multiple of 128");
    if (c.layers < 1 || c.vocab < 1 || c.max_pos < 3 || c.type_vocab < 1) return fail(RS_EARG, "bad config");
    if (!(c.heads_mask & (RS_HEAD_MLM | RS_HEAD_CLS | RS_HEAD_EMB))) return fail(RS_EARG, "heads_mask selects no head");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
        return fail(RS_EHIP, "no such HIP device");
    rs_model* m = new (std::nothrow) rs_model();
    if (!m) return fail(RS_ENOMEM, "alloc");
    m->cfg = c;
    m->device = device;
    if (c.precision != RS_PREC_FP16 && c.precision != RS_PREC_FP16X3) {
        delete m;
        return fail(RS_EARG, "unknown precision");
    }
    m->kx = c.precision == RS_PREC_FP16X3 ? 3 : 1;
    *out = m;
    return RS_OK;
}

int rs_model_set_tensor(rs_model* m, const char* key, const void* host_ptr, int dtype,
                        const int64_t* shape, int ndim) {
    if (!m || !key || !host_ptr || (ndim > 0 && !shape)) return fail(RS_EARG, "null argument");
    if (dtype != RS_DT_F32) return fail(RS_EUNSUP, "only float32 tensors are accepted");
    if (m->finalized) return fail(RS_ESTATE, "model already finalized");
    int64_t n = 1;
    for (int i = 0; i < ndim; ++i) {
        if (shape[i] < 0) return fail(RS_EARG, "negative dim");
        n *= shape[i];
    }
    std::vector<float> v((size_t)n);
    std::memcpy(v.data(), host_ptr, (size_t)n * 4);
    m->host[key] = std::move(v);
    return RS_OK;
}

int rs_model_finalize(rs_model* m) {
    if (!m) return fail(RS_EARG, "null model");
    if (m->finalized) return RS_OK;
    HIPTRY(hipSetDevice(m->device));
    const rs_bert_cfg& c = m->cfg;
    const size_t H = c.hidden, F = c.intermediate, V = c.vocab;
    std::string miss;
    const std::string e = "bert.embeddings.";
    auto* word = need(m, e + "word_embeddings.weight", V * H, &miss);
    auto* pos = need(m, e + "position_embeddings.weight", (size_t)c.max_pos * H, &miss);
    auto* typ = need(m, e + "token_type_embeddings.weight", (size_t)c.type_vocab * H, &miss);
    auto* eg = need(m, e + "LayerNorm.weight", H, &miss);
    auto* eb = need(m, e + "LayerNorm.bias", H, &miss);
    if (!miss.empty()) return fail(RS_ESTATE, "tensor " + miss);
    hipError_t err = hipSuccess;
#define UP32(dst, src, n) do { dst = upload_f32(m, *(src), (n), &err); if (err != hipSuccess) return fail(RS_EHIP, "upload"); } while (0)
#define UP16(dst, src, rp, cols) do {                                                                             \
        if (!fp16_range_ok(*(src)))                                                                             \
            return fail(RS_EUNSUP, std::string("weight '") + #src + "' has a value outside the fp16 range "    \
                                   "(|w| > 65504) of the GEMM operand images");                              \
        dst = upload_f16(m, *(src), (rp), (cols), m->kx, &err);                                                 \
        if (err != hipSuccess) return fail(RS_EHIP, "upload");                                                 \
    } while (0)
    UP32(m->word32, word, V * H);
    UP32(m->pos32, pos, (size_t)c.max_pos * H);
    UP32(m->type32, typ, H);     // token_type_ids are all 0 (modeling_bert.py:88-94)
    UP32(m->eg, eg, H);
    UP32(m->eb, eb, H);
    m->layers.resize(c.layers);
    // fp16x3: the split-operand GEMMs' interleaved weight images, when every projection weight
    // keeps 64 W_hi finite (x3s_range_ok); else the K-concatenated form runs every layer
    bool x3s_w = m->kx == 3;
    for (int i = 0; i < c.layers && x3s_w; ++i) {
        const std::string p = "bert.encoder.layer." + std::to_string(i) + ".";
        for (const char* k : {"attention.self.query.weight", "attention.self.key.weight", "attention.self.value.weight",
                              "attention.output.dense.weight", "intermediate.dense.weight", "output.dense.weight"}) {
            auto it = m->host.find(p + k);
            if (it != m->host.end() && !x3s_range_ok(it->second)) x3s_w = false;
        }
    }
#define UPIL(dst, src, cols) do { dst = upload_il(m, *(src), (cols), &err); if (err != hipSuccess) return fail(RS_EHIP, "upload"); } while (0)
    for (int i = 0; i < c.layers; ++i) {
        const std::string p = "bert.encoder.layer." + std::to_string(i) + ".";
        auto* wq = need(m, p + "attention.self.query.weight", H * H, &miss);
        auto* bq = need(m, p + "attention.self.query.bias", H, &miss);
        auto* wk = need(m, p + "attention.self.key.weight", H * H, &miss);
        auto* bk = need(m, p + "attention.self.key.bias", H, &miss);
        auto* wv = need(m, p + "attention.self.value.weight", H * H, &miss);
        auto* bv = need(m, p + "attention.self.value.bias", H, &miss);
        auto* wo = need(m, p + "attention.output.dense.weight", H * H, &miss);
        auto* bo = need(m, p + "attention.output.dense.bias", H, &miss);
        auto* g1 = need(m, p + "attention.output.LayerNorm.weight", H, &miss);
        auto* be1 = need(m, p + "attention.output.LayerNorm.bias", H, &miss);
        auto* w1 = need(m, p + "intermediate.dense.weight", F * H, &miss);
        auto* b1 = need(m, p + "intermediate.dense.bias", F, &miss);
        auto* w2 = need(m, p + "output.dense.weight", H * F, &miss);
        auto* b2 = need(m, p + "output.dense.bias", H, &miss);
        auto* g2 = need(m, p + "output.LayerNorm.weight", H, &miss);
        auto* be2 = need(m, p + "output.LayerNorm.bias", H, &miss);
        if (!miss.empty()) return fail(RS_ESTATE, "tensor " + miss);
        std::vector<float> wqkv, bqkv;
        wqkv.reserve(3 * H * H);
        for (auto* w : {wq, wk, wv}) wqkv.insert(wqkv.end(), w->begin(), w->end());
        for (auto* b : {bq, bk, bv}) bqkv.insert(bqkv.end(), b->begin(), b->end());
        Layer& L = m->layers[i];
        UP16(L.wqkv, &wqkv, 3 * H, H);
        UP32(L.bqkv, &bqkv, 3 * H);
        UP16(L.wo, wo, H, H);
        UP32(L.bo, bo, H);
        UP32(L.g1, g1, H);
        UP32(L.be1, be1, H);
        UP16(L.w1, w1, F, H);
        UP32(L.b1, b1, F);
        UP16(L.w2, w2, H, F);
        UP32(L.b2, b2, H);
        UP32(L.g2, g2, H);
        UP32(L.be2, be2, H);
        if (x3s_w) {
            UPIL(L.iqkv, &wqkv, H);
            UPIL(L.io, wo, H);
            UPIL(L.i1, w1, H);
            UPIL(L.i2, w2, F);
        }
    }
#undef UPIL
    m->x3s_w = x3s_w;
    if (c.heads_mask & RS_HEAD_MLM) {
        const std::string p = "cls.predictions.";
        auto* wt = need(m, p + "transform.dense.weight", H * H, &miss);
        auto* bt = need(m, p + "transform.dense.bias", H, &miss);
        auto* gt = need(m, p + "transform.LayerNorm.weight", H, &miss);
        auto* bet = need(m, p + "transform.LayerNorm.bias", H, &miss);
        auto* bd = need(m, p + "bias", V, &miss);
        if (!miss.empty()) return fail(RS_ESTATE, "tensor " + miss);
        // decoder weight is tied to the word embeddings (BertForMaskedLM._tied_weights_keys);
        // an explicitly provided cls.predictions.decoder.weight must equal it.
        auto it = m->host.find(p + "decoder.weight");
        const std::vector<float>* dec = word;
        if (it != m->host.end()) {
            if (it->second.size() != V * H) return fail(RS_EARG, "decoder.weight has wrong size");
            dec = &it->second;
        }
        m->vpad = (int)((V + 127) / 128 * 128);
        UP16(m->wt, wt, H, H);
        UP32(m->bt, bt, H);
        UP32(m->gt, gt, H);
        UP32(m->bet, bet, H);
        UP16(m->wdec, dec, (size_t)m->vpad, H);
        UP32(m->bdec, bd, (size_t)m->vpad);
    }
    if (c.heads_mask & RS_HEAD_CLS) {
        auto* wl = need(m, "linear.weight", H, &miss);
        auto* bl = need(m, "linear.bias", 1, &miss);
        if (!miss.empty()) return fail(RS_ESTATE, "tensor " + miss);
        UP32(m->wlin, wl, H);
        UP32(m->blin, bl, 1);
    }
#undef UP32
#undef UP16
    if (!m->call_done) HIPTRY(hipEventCreateWithFlags(&m->call_done, hipEventDisableTiming));
    m->host.clear();
    m->finalized = true;
    return RS_OK;
}

int rs_model_reserve(rs_model* m, int64_t max_rows) {
    if (!m) return fail(RS_EARG, "null model");
    if (!m->finalized) return fail(RS_ESTATE, "rs_model_finalize not called");
    return reserve_impl(m, max_rows);
}

int rs_pll_score(rs_model* m, const int32_t* d_tok, const int32_t* h_hyp_off, int32_t n_hyp,
                 double* d_pll, float* d_row_lp, void* stream) {
    if (!m || !h_hyp_off || n_hyp < 0 || (n_hyp > 0 && (!d_tok || !d_pll))) return fail(RS_EARG, "null argument");
    hipStream_t st = (hipStream_t)stream;
    if (n_hyp == 0) return RS_OK;
    HIPTRY(hipSetDevice(m->device));
    CALL_ORDER(m, st);
    SeqList sl;
    std::vector<int> hso(n_hyp + 1, 0);
    for (int h = 0; h < n_hyp; ++h) {
        const int o = h_hyp_off[h], T = h_hyp_off[h + 1] - o;
        if (T < 3) return fail(RS_EARG, "hypothesis " + std::to_string(h) + " has no word (T < 3)");
        for (int p = 1; p <= T - 2; ++p) sl.push(o, T, p, p, -1);   // do_job rows, p = mask_pos
        hso[h + 1] = (int)sl.size();
    }
    float* rows = d_row_lp;
    if (!rows) {
        HIPTRY(m->rowlp_tmp.ensure(sl.size() * 4));
        rows = m->rowlp_tmp.as<float>();
    }
    int* d_hso = nullptr;
    if (int r = run_all(m, st, d_tok, sl, MODE_MLM, rows, &hso, &d_hso)) return r;
    {
        ProfScope ps(m, st, RS_K_OTHER, 0);
        HIPTRY(launch_segsum_f64(rows, d_hso, n_hyp, d_pll, st));
    }
    return check_finite(m, st, rows, sl.size(), "masked-token log-probability");
}

int rs_masked_logprob(rs_model* m, const int32_t* d_ids, const int32_t* h_seq_off,
                      const int32_t* h_query, const int32_t* d_label, int32_t n_seq, float* d_out,
                      void* stream) {
    if (!m || !h_seq_off || !h_query || n_seq < 0 || (n_seq > 0 && (!d_ids || !d_label || !d_out)))
        return fail(RS_EARG, "null argument");
    if (n_seq == 0) return RS_OK;
    HIPTRY(hipSetDevice(m->device));
    CALL_ORDER(m, (hipStream_t)stream);
    SeqList sl;
    for (int s = 0; s < n_seq; ++s) {
        const int o = h_seq_off[s], T = h_seq_off[s + 1] - o;
        if (h_query[s] < 0 || h_query[s] >= T) return fail(RS_EARG, "query position outside its sequence");
        sl.push(o, T, -1, h_query[s], 0);   // ids already masked by the caller
    }
    if (int r = run_all(m, (hipStream_t)stream, d_ids, sl, MODE_MLM, d_out, nullptr, nullptr, d_label)) return r;
    return check_finite(m, (hipStream_t)stream, d_out, (size_t)n_seq, "masked-token log-probability");
}

int rs_cls_score(rs_model* m, const int32_t* d_tok, const int32_t* h_hyp_off, int32_t n_hyp,
                 float* d_out, void* stream) {
    if (!m || !h_hyp_off || n_hyp < 0 || (n_hyp > 0 && (!d_tok || !d_out))) return fail(RS_EARG, "null argument");
    if (n_hyp == 0) return RS_OK;
    HIPTRY(hipSetDevice(m->device));
    CALL_ORDER(m, (hipStream_t)stream);
    SeqList sl;
    for (int h = 0; h < n_hyp; ++h) {
        const int o = h_hyp_off[h], T = h_hyp_off[h + 1] - o;
        if (T < 1) return fail(RS_EARG, "empty hypothesis");
        sl.push(o, T, -1, 0, 0);      // query = [CLS] (RescoreBert/model.py:19)
    }
    if (int r = run_all(m, (hipStream_t)stream, d_tok, sl, MODE_CLS, d_out, nullptr, nullptr)) return r;
    return check_finite(m, (hipStream_t)stream, d_out, (size_t)n_hyp, "RescoreBert score");
}

int rs_token_embed(rs_model* m, const int32_t* d_tok, const int32_t* h_hyp_off, int32_t n_hyp,
                   void* d_emb, void* stream) {
    if (!m || !h_hyp_off || n_hyp < 0 || (n_hyp > 0 && (!d_tok || !d_emb))) return fail(RS_EARG, "null argument");
    if (n_hyp == 0) return RS_OK;
    HIPTRY(hipSetDevice(m->device));
    CALL_ORDER(m, (hipStream_t)stream);
    SeqList sl;
    for (int h = 0; h < n_hyp; ++h) {
        const int o = h_hyp_off[h], T = h_hyp_off[h + 1] - o;
        if (o < 0 || T < 1) return fail(RS_EARG, "hypothesis " + std::to_string(h) + " is empty");
        sl.push(o, T, -1, 0, 0);
    }
    m->emb_dst = (f16*)d_emb;
    const int r = run_all(m, (hipStream_t)stream, d_tok, sl, MODE_EMB, nullptr, nullptr, nullptr);
    m->emb_dst = nullptr;
    if (r) return r;
    // every token row of the hypotheses (contiguous from h_hyp_off[0]) is written
    const size_t W = (size_t)m->cfg.hidden * (m->kx == 3 ? 2 : 1);
    return check_finite(m, (hipStream_t)stream, (const f16*)d_emb + (size_t)h_hyp_off[0] * W,
                        (size_t)(h_hyp_off[n_hyp] - h_hyp_off[0]) * W, "token embedding");
}

int rs_bertscore_recall(rs_model* m, const int32_t* d_tok, const int32_t* h_hyp_off,
                        const int32_t* h_utt_off, int32_t n_utt, float* d_rmat, float* d_rmat0, void* stream) {
    if (!m || !h_hyp_off || !h_utt_off || n_utt < 0 || (n_utt > 0 && (!d_tok || !d_rmat)))
        return fail(RS_EARG, "null argument");
    if (n_utt == 0) return RS_OK;
    if (h_utt_off[0] != 0) return fail(RS_EARG, "utt_off[0] must be 0");
    const int n_hyp = h_utt_off[n_utt];
    for (int u = 0; u < n_utt; ++u)
        if (h_utt_off[u + 1] < h_utt_off[u]) return fail(RS_EARG, "utt_off not ascending");
    if (h_hyp_off[0] != 0) return fail(RS_EARG, "hyp_off[0] must be 0");
    for (int h = 0; h < n_hyp; ++h)
        if (h_hyp_off[h + 1] - h_hyp_off[h] < 2)
            return fail(RS_EARG, "hypothesis " + std::to_string(h) + " has fewer than 2 tokens ([CLS] [SEP])");
    hipStream_t st = (hipStream_t)stream;
    HIPTRY(hipSetDevice(m->device));
    CALL_ORDER(m, st);
    const int H = m->cfg.hidden;
    const size_t n_tok = (size_t)h_hyp_off[n_hyp];
    const bool two = m->kx == 3;                 // fp16x3: two-part embeddings, split-operand cosines
    const int COLS = bertscore_cols(two);
    HIPTRY(m->emb.ensure(std::max<size_t>(n_tok, 1) * H * 2 * (two ? 2 : 1)));
    if (int r = rs_token_embed(m, d_tok, h_hyp_off, n_hyp, m->emb.p, stream)) return r;
    // plan: runs of whole ref hypotheses fitting one COLS-column tile (a longer one alone)
    std::vector<int> items;
    std::vector<long long> moff(n_utt + 1, 0);
    for (int u = 0; u < n_utt; ++u) {
        const int h0 = h_utt_off[u], n = h_utt_off[u + 1] - h0;
        moff[u + 1] = moff[u] + (long long)n * n;
        for (int j = 0; j < n;) {
            int j1 = j + 1, cols = h_hyp_off[h0 + j + 1] - h_hyp_off[h0 + j];
            while (cols <= COLS && j1 < n && cols + h_hyp_off[h0 + j1 + 1] - h_hyp_off[h0 + j1] <= COLS) {
                cols += h_hyp_off[h0 + j1 + 1] - h_hyp_off[h0 + j1];
                ++j1;
            }
            items.insert(items.end(), {u, j, j1, 0});
            j = j1;
        }
    }
    const int n_items = (int)(items.size() / 4);
    // one upload: items | mat_off (int64) | hyp_off | utt_off
    const size_t w_items = items.size(), w_moff = 2 * (size_t)(n_utt + 1);
    const size_t n_int = w_items + w_moff + (size_t)(n_hyp + 1) + (size_t)(n_utt + 1);
    if (m->plan_done) HIPTRY(hipEventSynchronize(m->plan_done));
    if (n_int > m->pinned_plan_cap) {
        if (m->pinned_plan) (void)hipHostFree(m->pinned_plan);
        m->pinned_plan = nullptr;
        m->pinned_plan_cap = 0;
        HIPTRY(hipHostMalloc((void**)&m->pinned_plan, n_int * 4, hipHostMallocDefault));
        m->pinned_plan_cap = n_int;
    }
    int* p = m->pinned_plan;
    std::memcpy(p, items.data(), w_items * 4);
    std::memcpy(p + w_items, moff.data(), w_moff * 4);
    std::memcpy(p + w_items + w_moff, h_hyp_off, (size_t)(n_hyp + 1) * 4);
    std::memcpy(p + w_items + w_moff + n_hyp + 1, h_utt_off, (size_t)(n_utt + 1) * 4);
    HIPTRY(m->plan.ensure(n_int * 4));
    HIPTRY(hipMemcpyAsync(m->plan.p, p, n_int * 4, hipMemcpyHostToDevice, st));
    if (!m->plan_done) HIPTRY(hipEventCreateWithFlags(&m->plan_done, hipEventDisableTiming));
    HIPTRY(hipEventRecord(m->plan_done, st));
    int* d = m->plan.as<int>();
    ProfScope ps(m, st, RS_K_OTHER, 0);
    HIPTRY(launch_bertscore_recall(m->emb.as<f16>(), H, d + w_items + w_moff, d + w_items + w_moff + n_hyp + 1,
                                   (const long long*)(d + w_items), (const int4*)d, n_items, d_rmat, d_rmat0, st, two));
    return RS_OK;
}

int rs_model_set_sync_check(rs_model* m, int on) {
    if (!m) return fail(RS_EARG, "null model");
    m->sync_check = on != 0;
    return RS_OK;
}

int rs_check(rs_model* m, void* stream) {
    if (!m) return fail(RS_EARG, "null model");
    HIPTRY(hipSetDevice(m->device));
    CALL_ORDER(m, (hipStream_t)stream);
    return report_flags(m, (hipStream_t)stream, "scores");
}

int rs_profile_enable(rs_model* m, int on) {
    if (!m) return fail(RS_EARG, "null model");
    prof_collect(m);
    m->prof = on != 0;
    for (int k = 0; k < RS_K_COUNT; ++k) m->prof_ms[k] = 0, m->prof_n[k] = 0, m->prof_flops[k] = 0;
    return RS_OK;
}

int rs_profile_read(rs_model* m, int kind, double* ms, int64_t* launches, double* flops) {
    if (!m || kind < 0 || kind >= RS_K_COUNT) return fail(RS_EARG, "bad argument");
    prof_collect(m);
    if (ms) *ms = m->prof_ms[kind];
    if (launches) *launches = m->prof_n[kind];
    if (flops) *flops = m->prof_flops[kind];
    return RS_OK;
}

void rs_model_destroy(rs_model* m) {
    if (!m) return;
    (void)hipSetDevice(m->device);
    (void)hipDeviceSynchronize();
    for (void* p : m->allocs) (void)hipFree(p);
    for (DevBuf* b : {&m->xst, &m->xst1, &m->h16, &m->t32, &m->qkv, &m->ctx, &m->inter, &m->ctxq, &m->resq,
                      &m->tq32, &m->hq32, &m->hq16, &m->interq, &m->lab, &m->llog, &m->part,
                      &m->rowlp_tmp, &m->meta, &m->hypoff, &m->emb, &m->plan, &m->flag, &m->lnx, &m->lncnt,
                      &m->lnerr})
        b->release();
    if (m->pinned) (void)hipHostFree(m->pinned);
    if (m->pinned_plan) (void)hipHostFree(m->pinned_plan);
    if (m->pinned_flag) (void)hipHostFree(m->pinned_flag);
    if (m->plan_done) (void)hipEventDestroy(m->plan_done);
    if (m->upload_done) (void)hipEventDestroy(m->upload_done);
    if (m->call_done) (void)hipEventDestroy(m->call_done);
    for (hipEvent_t e : m->ev_pool) (void)hipEventDestroy(e);
    delete m;
}

}  // extern "C"

// shared error slot for the other C-ABI translation units (train_api.hip)
int rs_fail(int code, const std::string& msg) { return fail(code, msg); }
