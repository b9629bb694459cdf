// C-ABI trainer (include/rescore.h, rs_trainer_*): RescoreBert distillation training
// (RescoreBert/main.py:104-229 — MD / MD_MWER / MD_MWED) on the GPU.
//
// One step = forward over the batch's hypotheses with every activation the backward needs
// saved (ragged token rows, no padding), the loss and its gradient w.r.t. the CLS scores,
// the backward through the head, the encoder layers and the embeddings, then one
// torch.optim.AdamW update.  Parameters, gradients and Adam moments are single flat fp32
// buffers (one AdamW launch); the fused Q|K|V weight is the contiguous [q; k; v] range of
// the three HF tensors.  GEMMs: tr_sgemm (k_sgemm.hip: f32-input MFMA, exact fp32, split-K
// through an ordered workspace sum — deterministic); RS_TRAIN_ROCBLAS=1 routes them to rocBLAS
// sgemm instead (atomics disabled), kept as the timing / numerics baseline.
// All other ops: k_train.hip.  Dropout (BERT's train mode, train.h TrDrop): hidden dropout after
// the embedding LayerNorm and on both residual branches, attention-probability dropout; the keep
// bits are counter-based draws keyed by (dropout_seed, the trainer's dropout-step counter), so a
// step is bitwise reproducible and the backward recomputes the mask.
#include <algorithm>
#include <map>
#include <string>
#include <vector>
#include <cstring>
#include <cmath>
#include <cstdlib>

#include <rocblas/rocblas.h>

#include "common.h"
#include "train.h"

int rs_fail(int code, const std::string& msg);

namespace {

#define TRY_HIP(expr)                                                                       \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) return rs_fail(RS_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)
#define TRY_BLAS(expr)                                                                      \
    do {                                                                                    \
        rocblas_status s_ = (expr);                                                         \
        if (s_ != rocblas_status_success)                                                   \
            return rs_fail(RS_EHIP, std::string(#expr) + ": " + rocblas_status_to_string(s_)); \
    } while (0)

struct Buf {
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
    float* f() const { return (float*)p; }
};

struct TLayer {
    size_t wqkv, bqkv, wo, bo, g1, be1, w1, b1, w2, b2, g2, be2;
};

}  // namespace

struct rs_trainer {
    rs_bert_cfg cfg{};
    int device = 0;
    bool finalized = false;
    rocblas_handle blas = nullptr;
    bool use_rocblas = false;                                 // RS_TRAIN_ROCBLAS=1 (baseline)
    std::map<std::string, std::pair<size_t, size_t>> table;   // HF key -> (offset, numel) in floats
    std::vector<float> host;                                  // staged parameters until finalize
    std::vector<char> set;                                    // per table entry: provided?
    size_t n_params = 0;
    size_t o_word = 0, o_pos = 0, o_type = 0, o_eg = 0, o_eb = 0, o_wl = 0, o_bl = 0;
    size_t o_wt = 0, o_bt = 0, o_tg = 0, o_tb = 0, o_db = 0;   // MLM head (decoder tied to o_word)
    std::vector<TLayer> lay;
    Buf P, G, M1, V1;       // parameters, gradients, Adam moments
    Buf act, grad, meta, small, ws;   // ws: split-K partials of tr_sgemm
    long long step = 0;
    uint64_t drop_step = 0;         // dropout-step counter (key of the next dropout-active step)
    std::vector<int> h_tok, h_meta;
};

namespace {

size_t add_tensor(rs_trainer* t, const std::string& key, size_t n) {
    size_t off = (t->n_params + 63) / 64 * 64;
    t->table[key] = {off, n};
    t->n_params = off + n;
    return off;
}

// rocBLAS baseline (RS_TRAIN_ROCBLAS=1): the same three forms, column-major arguments
rocblas_status blas_nt(rocblas_handle h, int M, int N, int K, const float* X, const float* W, float* Y, float beta) {
    const float one = 1.0f;
    return rocblas_sgemm(h, rocblas_operation_transpose, rocblas_operation_none, N, M, K, &one, W, K, X, K, &beta, Y, N);
}
rocblas_status blas_nn(rocblas_handle h, int M, int N, int K, const float* dY, const float* W, float* dX, float beta) {
    const float one = 1.0f;
    return rocblas_sgemm(h, rocblas_operation_none, rocblas_operation_none, K, M, N, &one, W, K, dY, N, &beta, dX, K);
}
rocblas_status blas_tn(rocblas_handle h, int M, int N, int K, const float* dY, const float* X, float* dW, float beta) {
    const float one = 1.0f;
    return rocblas_sgemm(h, rocblas_operation_none, rocblas_operation_transpose, K, N, M, &one, X, K, dY, N, &beta, dW, K);
}

#define TRY_SG(expr)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) return rs_fail(RS_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define RS_TRY(expr)                     \
    do {                                 \
        if (int r_ = (expr)) return r_;  \
    } while (0)

// row-major Y[M, N] = X[M, K] . W[N, K]^T (+ beta Y)
int gemm_nt(rs_trainer* t, hipStream_t st, int M, int N, int K, const float* X, const float* W, float* Y, float beta) {
    if (t->use_rocblas) {
        TRY_BLAS(blas_nt(t->blas, M, N, K, X, W, Y, beta));
        return RS_OK;
    }
    TRY_SG(tr_sgemm(M, N, K, X, K, true, W, K, true, Y, N, beta != 0.f, t->ws.f(), t->ws.bytes / 4, st));
    return RS_OK;
}
// row-major dX[M, K] = dY[M, N] . W[N, K] (+ beta dX)
int gemm_nn(rs_trainer* t, hipStream_t st, int M, int N, int K, const float* dY, const float* W, float* dX, float beta) {
    if (t->use_rocblas) {
        TRY_BLAS(blas_nn(t->blas, M, N, K, dY, W, dX, beta));
        return RS_OK;
    }
    TRY_SG(tr_sgemm(M, K, N, dY, N, true, W, K, false, dX, K, beta != 0.f, t->ws.f(), t->ws.bytes / 4, st));
    return RS_OK;
}
// row-major dW[N, K] = dY[M, N]^T . X[M, K] (+ beta dW)
int gemm_tn(rs_trainer* t, hipStream_t st, int M, int N, int K, const float* dY, const float* X, float* dW, float beta) {
    if (t->use_rocblas) {
        TRY_BLAS(blas_tn(t->blas, M, N, K, dY, X, dW, beta));
        return RS_OK;
    }
    TRY_SG(tr_sgemm(N, K, M, dY, N, false, X, K, false, dW, K, beta != 0.f, t->ws.f(), t->ws.bytes / 4, st));
    return RS_OK;
}

// split-K workspace for every GEMM shape of a step over M token rows (forward, dgrad, wgrad of
// each Linear; the MLM head's transform and tied decoder)
size_t sgemm_ws_floats(const rs_bert_cfg& c, int M) {
    const int H = c.hidden, F = c.intermediate, V = c.heads_mask == RS_HEAD_MLM ? c.vocab : H;
    size_t w = 0;
    for (int n : {3 * H, H, F, V})
        for (int k : {H, F}) {
            w = std::max(w, tr_sgemm_ws_floats(M, n, k));   // forward (M, n, k)
            w = std::max(w, tr_sgemm_ws_floats(M, k, n));   // dgrad   (M, k, n)
            w = std::max(w, tr_sgemm_ws_floats(n, k, M));   // wgrad   (n, k, M)
        }
    return w;
}

}  // namespace

extern "C" {

int rs_trainer_create(const rs_bert_cfg* cfg, int device, rs_trainer** out) {
    if (!cfg || !out) return rs_fail(RS_EARG, "null argument");
    const rs_bert_cfg& c = *cfg;
    if (c.hidden <= 0 || c.hidden % 256 || c.hidden > 1024) return rs_fail(RS_EUNSUP, "hidden must be 256/512/768/1024");
    if (c.heads <= 0 || c.hidden / c.heads != 64 || c.hidden % c.heads) return rs_fail(RS_EUNSUP, "head_dim must be 64");
    if (c.intermediate <= 0 || c.intermediate % 4) return rs_fail(RS_EUNSUP, "intermediate must be a multiple of 4");
    if (c.layers < 1 || c.vocab < 1 || c.max_pos < 3 || c.type_vocab < 1) return rs_fail(RS_EARG, "bad config");
    if (c.heads_mask != RS_HEAD_CLS && c.heads_mask != RS_HEAD_MLM)
        return rs_fail(RS_EUNSUP, "the trainer takes one head: RS_HEAD_CLS (RescoreBert) or RS_HEAD_MLM (MLM fine-tuning)");
    if (c.heads_mask == RS_HEAD_MLM && c.vocab % 4) return rs_fail(RS_EUNSUP, "MLM training needs vocab % 4 == 0");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return rs_fail(RS_EHIP, "no such HIP device");
    rs_trainer* t = new (std::nothrow) rs_trainer();
    if (!t) return rs_fail(RS_ENOMEM, "alloc");
    t->cfg = c;
    t->device = device;
    const size_t H = c.hidden, F = c.intermediate, V = c.vocab;
    const std::string e = "bert.embeddings.";
    t->o_word = add_tensor(t, e + "word_embeddings.weight", V * H);
    t->o_pos = add_tensor(t, e + "position_embeddings.weight", (size_t)c.max_pos * H);
    t->o_type = add_tensor(t, e + "token_type_embeddings.weight", (size_t)c.type_vocab * H);
    t->o_eg = add_tensor(t, e + "LayerNorm.weight", H);
    t->o_eb = add_tensor(t, e + "LayerNorm.bias", H);
    t->lay.resize(c.layers);
    for (int i = 0; i < c.layers; ++i) {
        const std::string p = "bert.encoder.layer." + std::to_string(i) + ".";
        TLayer& L = t->lay[i];
        L.wqkv = add_tensor(t, p + "attention.self.query.weight", H * H);     // H*H % 64 == 0: contiguous
        add_tensor(t, p + "attention.self.key.weight", H * H);
        add_tensor(t, p + "attention.self.value.weight", H * H);
        L.bqkv = add_tensor(t, p + "attention.self.query.bias", H);
        add_tensor(t, p + "attention.self.key.bias", H);
        add_tensor(t, p + "attention.self.value.bias", H);
        L.wo = add_tensor(t, p + "attention.output.dense.weight", H * H);
        L.bo = add_tensor(t, p + "attention.output.dense.bias", H);
        L.g1 = add_tensor(t, p + "attention.output.LayerNorm.weight", H);
        L.be1 = add_tensor(t, p + "attention.output.LayerNorm.bias", H);
        L.w1 = add_tensor(t, p + "intermediate.dense.weight", F * H);
        L.b1 = add_tensor(t, p + "intermediate.dense.bias", F);
        L.w2 = add_tensor(t, p + "output.dense.weight", H * F);
        L.b2 = add_tensor(t, p + "output.dense.bias", H);
        L.g2 = add_tensor(t, p + "output.LayerNorm.weight", H);
        L.be2 = add_tensor(t, p + "output.LayerNorm.bias", H);
    }
    if (c.heads_mask == RS_HEAD_CLS) {
        t->o_wl = add_tensor(t, "linear.weight", H);
        t->o_bl = add_tensor(t, "linear.bias", 1);
    } else {
        const std::string p = "cls.predictions.";
        t->o_wt = add_tensor(t, p + "transform.dense.weight", H * H);
        t->o_bt = add_tensor(t, p + "transform.dense.bias", H);
        t->o_tg = add_tensor(t, p + "transform.LayerNorm.weight", H);
        t->o_tb = add_tensor(t, p + "transform.LayerNorm.bias", H);
        t->o_db = add_tensor(t, p + "bias", V);
    }
    t->n_params = (t->n_params + 63) / 64 * 64;
    t->host.assign(t->n_params, 0.0f);
    t->set.assign(t->table.size(), 0);
    *out = t;
    return RS_OK;
}

int rs_trainer_set_tensor(rs_trainer* t, const char* key, const void* host_ptr, int dtype, const int64_t* shape,
                          int ndim) {
    if (!t || !key || !host_ptr || (ndim > 0 && !shape)) return rs_fail(RS_EARG, "null argument");
    if (dtype != RS_DT_F32) return rs_fail(RS_EUNSUP, "only float32 tensors are accepted");
    if (t->finalized) return rs_fail(RS_ESTATE, "trainer already finalized");
    const std::string k(key);
    if (k.rfind("bert.pooler.", 0) == 0) return RS_OK;   // RescoreBert never uses the pooler output: no gradient
    // tied to the word embeddings / to cls.predictions.bias (BertForMaskedLM._tied_weights_keys)
    if (k == "cls.predictions.decoder.weight" || k == "cls.predictions.decoder.bias") return RS_OK;
    auto it = t->table.find(k);
    if (it == t->table.end()) return rs_fail(RS_EARG, "unknown tensor " + k);
    int64_t n = 1;
    for (int i = 0; i < ndim; ++i) n *= shape[i];
    if ((size_t)n != it->second.second) return rs_fail(RS_EARG, "tensor " + k + " has the wrong size");
    std::memcpy(t->host.data() + it->second.first, host_ptr, (size_t)n * 4);
    t->set[std::distance(t->table.begin(), it)] = 1;
    return RS_OK;
}

int rs_trainer_finalize(rs_trainer* t) {
    if (!t) return rs_fail(RS_EARG, "null trainer");
    if (t->finalized) return RS_OK;
    size_t i = 0;
    for (auto& kv : t->table) {
        if (!t->set[i++]) return rs_fail(RS_ESTATE, "tensor " + kv.first + " (missing)");
    }
    TRY_HIP(hipSetDevice(t->device));
    const size_t bytes = t->n_params * 4;
    TRY_HIP(t->P.ensure(bytes));
    TRY_HIP(t->G.ensure(bytes));
    TRY_HIP(t->M1.ensure(bytes));
    TRY_HIP(t->V1.ensure(bytes));
    TRY_HIP(hipMemcpy(t->P.p, t->host.data(), bytes, hipMemcpyHostToDevice));
    TRY_HIP(hipMemset(t->G.p, 0, bytes));
    TRY_HIP(hipMemset(t->M1.p, 0, bytes));
    TRY_HIP(hipMemset(t->V1.p, 0, bytes));
    TRY_BLAS(rocblas_create_handle(&t->blas));
    TRY_BLAS(rocblas_set_atomics_mode(t->blas, rocblas_atomics_not_allowed));
    {
        const char* v = getenv("RS_TRAIN_ROCBLAS");
        t->use_rocblas = v && v[0] == '1';
    }
    t->host.clear();
    t->host.shrink_to_fit();
    t->finalized = true;
    return RS_OK;
}

static int copy_out(rs_trainer* t, const Buf& b, const char* key, void* host_out, int64_t numel) {
    if (!t || !key || !host_out) return rs_fail(RS_EARG, "null argument");
    if (!t->finalized) return rs_fail(RS_ESTATE, "rs_trainer_finalize not called");
    auto it = t->table.find(key);
    if (it == t->table.end()) return rs_fail(RS_EARG, std::string("unknown tensor ") + key);
    if ((size_t)numel != it->second.second) return rs_fail(RS_EARG, std::string("tensor ") + key + " has a different size");
    TRY_HIP(hipSetDevice(t->device));
    TRY_HIP(hipDeviceSynchronize());
    TRY_HIP(hipMemcpy(host_out, b.f() + it->second.first, (size_t)numel * 4, hipMemcpyDeviceToHost));
    return RS_OK;
}

int rs_trainer_get_tensor(rs_trainer* t, const char* key, void* host_out, int64_t numel) {
    return copy_out(t, t ? t->P : Buf{}, key, host_out, numel);
}

int rs_trainer_get_grad(rs_trainer* t, const char* key, void* host_out, int64_t numel) {
    return copy_out(t, t ? t->G : Buf{}, key, host_out, numel);
}

}  // extern "C"

namespace {

// One step's ragged batch: metadata on the device, saved activations, gradient scratch.
struct StepCtx {
    rs_trainer* t;
    hipStream_t st;
    int M = 0, S = 0, tmax = 0, n_uniq = 0;
    const int* dm = nullptr;
    const long long* pofs = nullptr;
    const int* seq = nullptr;
    size_t i_tok = 0, i_pos = 0, i_aux = 0, i_utok = 0, i_toff = 0, i_ord = 0, i_klen = 0;
    float* x0 = nullptr;
    float2* st0 = nullptr;
    struct LA { float *hin, *qkv, *P, *ctx, *x1, *h1, *pre, *act, *x2; float2 *st1, *st2; };
    std::vector<LA> la;
    float *dA = nullptr, *dB = nullptr, *dQKV = nullptr, *dF = nullptr, *part = nullptr, *tail = nullptr;
    // MLM head (RS_HEAD_MLM): transform pre-GELU / GELU out (pre-LN) / LN out, stats, logits
    float *tpre = nullptr, *tx = nullptr, *th = nullptr, *logits = nullptr;
    float2* tst = nullptr;
    // dropout of this step (train mode: update >= 0 and p > 0)
    uint32_t seed = 0, th_hidden = 0, th_attn = 0;
    uint64_t dstep = 0;
    float sc_hidden = 1.f, sc_attn = 1.f;
    TrDrop drop(uint32_t site, bool attn) const {
        TrDrop d;
        d.seed = seed;
        d.step = (uint32_t)dstep;
        d.step_hi = (uint32_t)(dstep >> 32);
        d.site = site;
        d.thresh = attn ? th_attn : th_hidden;
        d.scale = attn ? sc_attn : sc_hidden;
        return d;
    }
};

uint32_t drop_thresh(float p) { return p <= 0.f ? 0u : (uint32_t)std::min(4294967295.0, (double)p * 4294967296.0); }

// train mode (the reference's model.train() under grad_update) with p > 0: this step's key
int set_dropout(StepCtx& c, const rs_train_opts* o) {
    if (!(o->hidden_dropout >= 0.f && o->hidden_dropout < 1.f && o->attn_dropout >= 0.f && o->attn_dropout < 1.f))
        return rs_fail(RS_EARG, "dropout probabilities must be in [0, 1)");
    if (o->update < 0 || (o->hidden_dropout == 0.f && o->attn_dropout == 0.f)) return RS_OK;   // eval mode
    c.seed = o->dropout_seed;
    c.dstep = c.t->drop_step++;
    c.th_hidden = drop_thresh(o->hidden_dropout);
    c.th_attn = drop_thresh(o->attn_dropout);
    c.sc_hidden = (float)(1.0 / (1.0 - (double)o->hidden_dropout));
    c.sc_attn = (float)(1.0 / (1.0 - (double)o->attn_dropout));
    return RS_OK;
}

// host metadata + buffers.  aux: extra int32 array uploaded with the metadata (utt_off);
// h_klen (nullable): per-sequence key lengths (padded-batch rows, rs_train_step_mlm).
int prepare(StepCtx& c, const int32_t* d_tok, const int32_t* h_off, int n_seq, const std::vector<int>& aux,
            const int32_t* h_klen = nullptr) {
    rs_trainer* t = c.t;
    const rs_bert_cfg& cf = t->cfg;
    const int H = cf.hidden, F = cf.intermediate, nh = cf.heads, NL = cf.layers;
    if (n_seq <= 0 || h_off[0] != 0) return rs_fail(RS_EARG, "empty batch or offsets not starting at 0");
    c.S = n_seq;
    c.M = h_off[n_seq];
    for (int s = 0; s < n_seq; ++s) {
        const int T = h_off[s + 1] - h_off[s];
        if (T < 1) return rs_fail(RS_EARG, "empty sequence");
        c.tmax = std::max(c.tmax, T);
    }
    if (c.tmax > cf.max_pos) return rs_fail(RS_EUNSUP, "sequence longer than max_position_embeddings");
    if (c.tmax > 128) return rs_fail(RS_EUNSUP, "training sequences are limited to 128 tokens");
    if (h_klen)
        for (int s = 0; s < n_seq; ++s)
            if (h_klen[s] < 1 || h_klen[s] > h_off[s + 1] - h_off[s])
                return rs_fail(RS_EARG, "key length outside 1..row length");
    const int M = c.M, S = c.S;
    hipStream_t st = c.st;
    TRY_HIP(hipSetDevice(t->device));
    TRY_BLAS(rocblas_set_stream(t->blas, st));
    t->h_tok.resize(M);
    TRY_HIP(hipMemcpyAsync(t->h_tok.data(), d_tok, (size_t)M * 4, hipMemcpyDeviceToHost, st));
    TRY_HIP(hipStreamSynchronize(st));
    std::vector<int> row_pos(M), order(M);
    for (int s = 0; s < S; ++s)
        for (int r = h_off[s]; r < h_off[s + 1]; ++r) row_pos[r] = r - h_off[s];
    for (int r = 0; r < M; ++r) {
        order[r] = r;
        t->h_tok[r] = std::min(std::max(t->h_tok[r], 0), cf.vocab - 1);
    }
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return t->h_tok[a] < t->h_tok[b]; });
    std::vector<int> utok, toff;
    for (int k = 0; k < M; ++k)
        if (k == 0 || t->h_tok[order[k]] != t->h_tok[order[k - 1]]) {
            utok.push_back(t->h_tok[order[k]]);
            toff.push_back(k);
        }
    toff.push_back(M);
    c.n_uniq = (int)utok.size();
    std::vector<long long> pofs(S + 1, 0);
    for (int s = 0; s < S; ++s) {
        const long long T = h_off[s + 1] - h_off[s];
        pofs[s + 1] = pofs[s] + (long long)nh * T * T;
    }
    // int layout: pofs (int64) | row_tok | row_pos | seq_off | aux | utok | toff | order | klen
    std::vector<int>& hm = t->h_meta;
    hm.assign(2 * (S + 1), 0);
    std::memcpy(hm.data(), pofs.data(), (S + 1) * 8);
    c.i_tok = hm.size();
    hm.insert(hm.end(), t->h_tok.begin(), t->h_tok.end());
    c.i_pos = hm.size();
    hm.insert(hm.end(), row_pos.begin(), row_pos.end());
    const size_t i_seq = hm.size();
    hm.insert(hm.end(), h_off, h_off + S + 1);
    c.i_aux = hm.size();
    hm.insert(hm.end(), aux.begin(), aux.end());
    c.i_utok = hm.size();
    hm.insert(hm.end(), utok.begin(), utok.end());
    c.i_toff = hm.size();
    hm.insert(hm.end(), toff.begin(), toff.end());
    c.i_ord = hm.size();
    hm.insert(hm.end(), order.begin(), order.end());
    c.i_klen = 0;
    if (h_klen) {
        c.i_klen = hm.size();
        hm.insert(hm.end(), h_klen, h_klen + S);
    }
    TRY_HIP(t->meta.ensure(hm.size() * 4));
    TRY_HIP(hipMemcpyAsync(t->meta.p, hm.data(), hm.size() * 4, hipMemcpyHostToDevice, st));
    c.dm = (const int*)t->meta.p;
    c.pofs = (const long long*)c.dm;
    c.seq = c.dm + i_seq;

    const bool mlm = cf.heads_mask == RS_HEAD_MLM;
    // every region starts on a 256-byte boundary (an odd row count M would otherwise leave the
    // tensors after the float2 statistics 8-byte aligned under float4 accesses and rocBLAS)
    auto al = [](size_t n) { return (n + 63) & ~(size_t)63; };
    const size_t MH = al((size_t)M * H), MF = al((size_t)M * F), M2 = al((size_t)M * 2), PS = al((size_t)pofs[S]);
    const size_t QKV = al((size_t)M * 3 * H);
    const size_t MV = mlm ? al((size_t)M * cf.vocab) : 0;
    const size_t per_layer = MH + QKV + PS + MH + MH + M2 + MH + 2 * MF + MH + M2;
    const size_t n_head = mlm ? 3 * MH + M2 + MV : 0;
    const size_t n_act = MH + M2 + NL * per_layer + MH + n_head;
    TRY_HIP(t->act.ensure(n_act * 4));
    const int widest = std::max(std::max(3 * H, F), mlm ? cf.vocab : 0);
    const size_t n_part = al(tr_colsum_scratch(M, widest) / 4);
    const size_t n_grad = 2 * MH + QKV + MF + n_part + 2 * (size_t)S + aux.size() + M + 64;
    TRY_HIP(t->grad.ensure(n_grad * 4));
    TRY_HIP(t->ws.ensure(std::max<size_t>(sgemm_ws_floats(cf, M), 64) * 4));
    float* A = t->act.f();
    c.x0 = A;
    c.st0 = (float2*)(c.x0 + MH);
    float* lbase = c.x0 + MH + M2;
    c.la.assign(NL + 1, StepCtx::LA{});
    for (int l = 0; l <= NL; ++l) {
        float* b = lbase + (size_t)l * per_layer;
        StepCtx::LA& a = c.la[l];
        a.hin = b;
        if (l == NL) break;
        a.qkv = b + MH;
        a.P = a.qkv + QKV;
        a.ctx = a.P + PS;
        a.x1 = a.ctx + MH;
        a.st1 = (float2*)(a.x1 + MH);
        a.h1 = a.x1 + MH + M2;
        a.pre = a.h1 + MH;
        a.act = a.pre + MF;
        a.x2 = a.act + MF;
        a.st2 = (float2*)(a.x2 + MH);
    }
    if (mlm) {
        c.tpre = c.la[NL].hin + MH;
        c.tx = c.tpre + MH;
        c.th = c.tx + MH;
        c.tst = (float2*)(c.th + MH);
        c.logits = c.th + MH + M2;
    }
    float* G = t->grad.f();
    c.dA = G;
    c.dB = c.dA + MH;
    c.dQKV = c.dB + MH;
    c.dF = c.dQKV + QKV;
    c.part = c.dF + MF;
    c.tail = c.part + n_part;        // per-sequence / per-row small arrays
    return RS_OK;
}

int encoder_forward(StepCtx& c) {
    rs_trainer* t = c.t;
    const rs_bert_cfg& cf = t->cfg;
    const int H = cf.hidden, F = cf.intermediate, nh = cf.heads, M = c.M;
    float* Pm = t->P.f();
    hipStream_t st = c.st;
    TRY_HIP(tr_embed_ln(c.dm + c.i_tok, c.dm + c.i_pos, M, cf.vocab, Pm + t->o_word, Pm + t->o_pos, Pm + t->o_type,
                        Pm + t->o_eg, Pm + t->o_eb, cf.ln_eps, H, c.x0, c.st0, c.la[0].hin, st, c.drop(0, false)));
    for (int l = 0; l < cf.layers; ++l) {
        const TLayer& L = t->lay[l];
        StepCtx::LA& a = c.la[l];
        RS_TRY(gemm_nt(t, st, M, 3 * H, H, a.hin, Pm + L.wqkv, a.qkv, 0.f));
        TRY_HIP(tr_bias(a.qkv, Pm + L.bqkv, M, 3 * H, st));
        TRY_HIP(tr_attn_fwd(a.qkv, c.seq, c.i_klen ? c.dm + c.i_klen : nullptr, c.pofs, c.S, c.tmax, H, nh, a.P,
                            a.ctx, st, c.drop(1 + 3 * l, true)));
        RS_TRY(gemm_nt(t, st, M, H, H, a.ctx, Pm + L.wo, a.x1, 0.f));
        TRY_HIP(tr_bias_res_ln(a.x1, Pm + L.bo, a.hin, M, Pm + L.g1, Pm + L.be1, cf.ln_eps, H, a.st1, a.h1, st,
                               c.drop(2 + 3 * l, false)));
        RS_TRY(gemm_nt(t, st, M, F, H, a.h1, Pm + L.w1, a.pre, 0.f));
        TRY_HIP(tr_bias_gelu(a.pre, Pm + L.b1, a.act, M, F, st));
        RS_TRY(gemm_nt(t, st, M, H, F, a.act, Pm + L.w2, a.x2, 0.f));
        TRY_HIP(tr_bias_res_ln(a.x2, Pm + L.b2, a.h1, M, Pm + L.g2, Pm + L.be2, cf.ln_eps, H, a.st2,
                               c.la[l + 1].hin, st, c.drop(3 + 3 * l, false)));
    }
    return RS_OK;
}

// from dA = d(final hidden) down to the embeddings; gradients written into t->G (zeroed by
// the caller before the head's backward)
int encoder_backward(StepCtx& c) {
    rs_trainer* t = c.t;
    const rs_bert_cfg& cf = t->cfg;
    const int H = cf.hidden, F = cf.intermediate, nh = cf.heads, M = c.M;
    const size_t MH = (size_t)M * H, MF = (size_t)M * F;
    float *Pm = t->P.f(), *Gm = t->G.f();
    float *dA = c.dA, *dB = c.dB, *dF = c.dF, *dQKV = c.dQKV, *part = c.part;
    hipStream_t st = c.st;
    for (int l = cf.layers - 1; l >= 0; --l) {
        const TLayer& L = t->lay[l];
        StepCtx::LA& a = c.la[l];
        TRY_HIP(tr_colsum_ln(dA, a.x2, a.st2, M, H, part, Gm + L.g2, Gm + L.be2, st));
        TRY_HIP(tr_ln_bwd(dA, a.x2, a.st2, Pm + L.g2, dB, M, H, st));              // dB = dx2
        // BertOutput dropout: the dense branch sees dx2 * mask * scale (in the free dQKV
        // buffer), the residual branch dx2 itself (dB, copied into dA below)
        const float* dBo = dB;
        if (c.th_hidden) {
            TRY_HIP(tr_dropout(dQKV, dB, (long long)MH, c.drop(3 + 3 * l, false), st));
            dBo = dQKV;
        }
        TRY_HIP(tr_colsum(dBo, nullptr, nullptr, M, H, 0, part, Gm + L.b2, 0, st));
        RS_TRY(gemm_tn(t, st, M, H, F, dBo, a.act, Gm + L.w2, 0.f));
        RS_TRY(gemm_nn(t, st, M, H, F, dBo, Pm + L.w2, dF, 0.f));                   // d act
        TRY_HIP(tr_gelu_bwd(dF, a.pre, (long long)MF, st));                         // d pre
        TRY_HIP(tr_colsum(dF, nullptr, nullptr, M, F, 0, part, Gm + L.b1, 0, st));
        RS_TRY(gemm_tn(t, st, M, F, H, dF, a.h1, Gm + L.w1, 0.f));
        TRY_HIP(hipMemcpyAsync(dA, dB, MH * 4, hipMemcpyDeviceToDevice, st));      // residual
        RS_TRY(gemm_nn(t, st, M, F, H, dF, Pm + L.w1, dA, 1.f));                     // dA = d h1
        TRY_HIP(tr_colsum_ln(dA, a.x1, a.st1, M, H, part, Gm + L.g1, Gm + L.be1, st));
        TRY_HIP(tr_ln_bwd(dA, a.x1, a.st1, Pm + L.g1, dB, M, H, st));              // dB = dx1
        // BertSelfOutput dropout: masked copy for the dense branch in the free dF buffer
        const float* dBs = dB;
        if (c.th_hidden) {
            TRY_HIP(tr_dropout(dF, dB, (long long)MH, c.drop(2 + 3 * l, false), st));
            dBs = dF;
        }
        TRY_HIP(tr_colsum(dBs, nullptr, nullptr, M, H, 0, part, Gm + L.bo, 0, st));
        RS_TRY(gemm_tn(t, st, M, H, H, dBs, a.ctx, Gm + L.wo, 0.f));
        RS_TRY(gemm_nn(t, st, M, H, H, dBs, Pm + L.wo, dA, 0.f));                    // dA = d ctx
        TRY_HIP(tr_attn_bwd(a.qkv, a.P, dA, c.seq, c.pofs, c.S, c.tmax, H, nh, dQKV, st, c.drop(1 + 3 * l, true)));
        TRY_HIP(tr_colsum(dQKV, nullptr, nullptr, M, 3 * H, 0, part, Gm + L.bqkv, 0, st));
        RS_TRY(gemm_tn(t, st, M, 3 * H, H, dQKV, a.hin, Gm + L.wqkv, 0.f));
        TRY_HIP(hipMemcpyAsync(dA, dB, MH * 4, hipMemcpyDeviceToDevice, st));      // residual
        RS_TRY(gemm_nn(t, st, M, 3 * H, H, dQKV, Pm + L.wqkv, dA, 1.f));             // dA = d h_in
    }
    // embedding dropout: d(LN output) = d h0 * mask * scale
    if (c.th_hidden) TRY_HIP(tr_dropout(dA, dA, (long long)MH, c.drop(0, false), st));
    TRY_HIP(tr_colsum_ln(dA, c.x0, c.st0, M, H, part, Gm + t->o_eg, Gm + t->o_eb, st));
    TRY_HIP(tr_ln_bwd(dA, c.x0, c.st0, Pm + t->o_eg, dB, M, H, st));                // dB = dx0
    // word embeddings: += (the tied MLM decoder already wrote its part)
    TRY_HIP(tr_word_grad(dB, c.dm + c.i_utok, c.dm + c.i_toff, c.dm + c.i_ord, c.n_uniq, H, Gm + t->o_word, st));
    TRY_HIP(tr_pos_grad(dB, c.seq, c.S, c.tmax, H, Gm + t->o_pos, st));
    TRY_HIP(tr_colsum(dB, nullptr, nullptr, M, H, 0, part, Gm + t->o_type, 0, st));  // token_type row 0
    return RS_OK;
}

int adamw(rs_trainer* t, const rs_train_opts* o, hipStream_t st) {
    if (o->update != 1) return RS_OK;
    t->step += 1;
    const double bc1 = 1.0 - std::pow((double)o->beta1, (double)t->step);
    const double bc2 = 1.0 - std::pow((double)o->beta2, (double)t->step);
    // python-float (double) scalars as torch computes them, cast to the fp32 tensor dtype
    const float decay = (float)(1.0 - (double)o->lr * (double)o->weight_decay);
    TRY_HIP(tr_adamw(t->P.f(), t->G.f(), t->M1.f(), t->V1.f(), (long long)t->n_params, decay,
                     (float)(1.0 - (double)o->beta1), o->beta2, (float)(1.0 - (double)o->beta2),
                     (float)((double)o->lr / bc1), (float)std::sqrt(bc2), o->eps, st));
    return RS_OK;
}

}  // namespace

extern "C" {

int rs_train_step_cls(rs_trainer* t, const int32_t* d_tok, const int32_t* h_hyp_off, int32_t n_hyp,
                      const int32_t* h_utt_off, int32_t n_utt, const float* d_target, const float* d_am,
                      const float* d_err, const rs_train_opts* o, float* d_scores, float* d_loss, void* stream) {
    if (!t || !h_hyp_off || !h_utt_off || !o || !d_loss || n_hyp <= 0 || n_utt <= 0 || !d_tok || !d_target)
        return rs_fail(RS_EARG, "null argument / empty batch");
    if (!t->finalized) return rs_fail(RS_ESTATE, "rs_trainer_finalize not called");
    if (t->cfg.heads_mask != RS_HEAD_CLS) return rs_fail(RS_ESTATE, "trainer has no RescoreBert head");
    if (o->loss < RS_LOSS_MD || o->loss > RS_LOSS_MWED) return rs_fail(RS_EARG, "unknown loss");
    if (o->loss != RS_LOSS_MD && (!d_am || !d_err)) return rs_fail(RS_EARG, "MWER/MWED need am scores and errors");
    if (h_utt_off[0] != 0 || h_utt_off[n_utt] != n_hyp) return rs_fail(RS_EARG, "utt_off must span 0..n_hyp");
    for (int u = 0; u < n_utt; ++u)
        if (h_utt_off[u + 1] < h_utt_off[u]) return rs_fail(RS_EARG, "utt_off not ascending");
    StepCtx c;
    c.t = t;
    c.st = (hipStream_t)stream;
    if (int r = set_dropout(c, o)) return r;
    if (int r = prepare(c, d_tok, h_hyp_off, n_hyp, std::vector<int>(h_utt_off, h_utt_off + n_utt + 1))) return r;
    if (int r = encoder_forward(c)) return r;
    const int H = t->cfg.hidden, S = c.S;
    float *Pm = t->P.f(), *Gm = t->G.f();
    float* sc = c.tail;
    float* dsc = sc + S;
    float* uloss = dsc + S;
    const float* hfin = c.la[t->cfg.layers].hin;
    hipStream_t st = c.st;
    TRY_HIP(tr_cls_fwd(hfin, c.seq, S, H, Pm + t->o_wl, Pm + t->o_bl, sc, st));
    if (d_scores) TRY_HIP(hipMemcpyAsync(d_scores, sc, (size_t)S * 4, hipMemcpyDeviceToDevice, st));
    TRY_HIP(tr_loss(sc, d_target, d_am, d_err, c.dm + c.i_aux, n_utt, S, o->loss, o->md_loss_weight, dsc, uloss,
                    d_loss, st));
    if (o->update < 0) {                      // loss only (the reference's dev pass)
        TRY_HIP(hipStreamSynchronize(st));
        return RS_OK;
    }
    TRY_HIP(hipMemsetAsync(Gm, 0, t->n_params * 4, st));
    TRY_HIP(hipMemsetAsync(c.dA, 0, (size_t)c.M * H * 4, st));
    TRY_HIP(tr_cls_bwd(dsc, hfin, c.seq, S, H, Pm + t->o_wl, c.dA, Gm + t->o_wl, Gm + t->o_bl, st));
    if (int r = encoder_backward(c)) return r;
    if (int r = adamw(t, o, st)) return r;
    TRY_HIP(hipStreamSynchronize(st));        // the metadata upload read t->h_meta
    if (tr_sgemm_failed()) return rs_fail(RS_EHIP, "a stream-K GEMM timed out waiting for a partial tile");
    return RS_OK;
}

int rs_train_step_mlm(rs_trainer* t, const int32_t* d_ids, const int32_t* h_seq_off, int32_t n_seq,
                      const int32_t* h_key_len, const int32_t* d_labels, const rs_train_opts* o, float* d_loss,
                      void* stream) {
    if (!t || !h_seq_off || !o || !d_loss || n_seq <= 0 || !d_ids || !d_labels)
        return rs_fail(RS_EARG, "null argument / empty batch");
    if (!t->finalized) return rs_fail(RS_ESTATE, "rs_trainer_finalize not called");
    if (t->cfg.heads_mask != RS_HEAD_MLM) return rs_fail(RS_ESTATE, "trainer has no MLM head");
    StepCtx c;
    c.t = t;
    c.st = (hipStream_t)stream;
    if (int r = set_dropout(c, o)) return r;
    if (int r = prepare(c, d_ids, h_seq_off, n_seq, {}, h_key_len)) return r;
    if (int r = encoder_forward(c)) return r;
    const rs_bert_cfg& cf = t->cfg;
    const int H = cf.hidden, V = cf.vocab, M = c.M;
    float *Pm = t->P.f(), *Gm = t->G.f();
    hipStream_t st = c.st;
    const float* hfin = c.la[cf.layers].hin;
    // BertOnlyMLMHead: transform (dense + GELU + LN), tied decoder + bias (modeling_bert.py:466-506)
    RS_TRY(gemm_nt(t, st, M, H, H, hfin, Pm + t->o_wt, c.tpre, 0.f));
    TRY_HIP(tr_bias_gelu(c.tpre, Pm + t->o_bt, c.tx, M, H, st));
    TRY_HIP(tr_bias_res_ln(c.tx, nullptr, nullptr, M, Pm + t->o_tg, Pm + t->o_tb, cf.ln_eps, H, c.tst, c.th, st));
    RS_TRY(gemm_nt(t, st, M, V, H, c.th, Pm + t->o_word, c.logits, 0.f));
    TRY_HIP(tr_bias(c.logits, Pm + t->o_db, M, V, st));
    float* rl = c.tail;
    TRY_HIP(tr_ce(c.logits, d_labels, M, V, rl, d_loss, st));       // logits <- dlogits
    if (o->update < 0) {                      // loss only (the reference's dev pass)
        TRY_HIP(hipStreamSynchronize(st));
        return RS_OK;
    }
    TRY_HIP(hipMemsetAsync(Gm, 0, t->n_params * 4, st));
    float* dT = c.dB;
    float* dT2 = c.dF;
    TRY_HIP(tr_colsum(c.logits, nullptr, nullptr, M, V, 0, c.part, Gm + t->o_db, 0, st));
    RS_TRY(gemm_tn(t, st, M, V, H, c.logits, c.th, Gm + t->o_word, 0.f));          // tied decoder part
    RS_TRY(gemm_nn(t, st, M, V, H, c.logits, Pm + t->o_word, dT, 0.f));
    TRY_HIP(tr_colsum_ln(dT, c.tx, c.tst, M, H, c.part, Gm + t->o_tg, Gm + t->o_tb, st));
    TRY_HIP(tr_ln_bwd(dT, c.tx, c.tst, Pm + t->o_tg, dT2, M, H, st));
    TRY_HIP(tr_gelu_bwd(dT2, c.tpre, (long long)M * H, st));
    TRY_HIP(tr_colsum(dT2, nullptr, nullptr, M, H, 0, c.part, Gm + t->o_bt, 0, st));
    RS_TRY(gemm_tn(t, st, M, H, H, dT2, hfin, Gm + t->o_wt, 0.f));
    RS_TRY(gemm_nn(t, st, M, H, H, dT2, Pm + t->o_wt, c.dA, 0.f));                  // dA = d hidden
    if (int r = encoder_backward(c)) return r;
    if (int r = adamw(t, o, st)) return r;
    TRY_HIP(hipStreamSynchronize(st));
    if (tr_sgemm_failed()) return rs_fail(RS_EHIP, "a stream-K GEMM timed out waiting for a partial tile");
    return RS_OK;
}

int rs_trainer_reset_optimizer(rs_trainer* t) {
    if (!t) return rs_fail(RS_EARG, "null trainer");
    if (!t->finalized) return rs_fail(RS_ESTATE, "rs_trainer_finalize not called");
    TRY_HIP(hipSetDevice(t->device));
    TRY_HIP(hipDeviceSynchronize());
    TRY_HIP(hipMemset(t->M1.p, 0, t->n_params * 4));
    TRY_HIP(hipMemset(t->V1.p, 0, t->n_params * 4));
    t->step = 0;
    return RS_OK;
}

int64_t rs_trainer_dropout_step(const rs_trainer* t) { return t ? (int64_t)t->drop_step : -1; }

int rs_trainer_set_dropout_step(rs_trainer* t, int64_t step) {
    if (!t || step < 0) return rs_fail(RS_EARG, "bad argument");
    t->drop_step = (uint64_t)step;
    return RS_OK;
}

int rs_dropout_keep(uint32_t seed, uint64_t step, uint32_t site, float p, int64_t n, uint8_t* d_keep, void* stream) {
    if (n < 0 || (n > 0 && !d_keep)) return rs_fail(RS_EARG, "null argument");
    if (!(p >= 0.f && p < 1.f)) return rs_fail(RS_EARG, "p must be in [0, 1)");
    TrDrop d;
    d.seed = seed;
    d.step = (uint32_t)step;
    d.step_hi = (uint32_t)(step >> 32);
    d.site = site;
    d.thresh = drop_thresh(p);
    TRY_HIP(tr_dropout_keep(d_keep, (long long)n, d, (hipStream_t)stream));
    return RS_OK;
}

void rs_trainer_destroy(rs_trainer* t) {
    if (!t) return;
    (void)hipSetDevice(t->device);
    (void)hipDeviceSynchronize();
    if (t->blas) (void)rocblas_destroy_handle(t->blas);
    for (Buf* b : {&t->P, &t->G, &t->M1, &t->V1, &t->act, &t->grad, &t->meta, &t->small, &t->ws}) b->release();
    delete t;
}

}  // extern "C"
