// Training kernels (k_train.hip) used by the trainer (train_api.hip).
//
// Distillation losses of RescoreBert training, as RescoreBert/main.py:104-147 computes them
// (groups g of consecutive hypotheses = the reference's reshape(-1, n_best)):
//   s_i = CLS score, t_i = mlm_pll_score, c_i = s_i + hyps_am_score_i, e_i = hyps_cer_i
//   MD      = sum_i (s_i - t_i)^2                                   (MSELoss(reduction="sum"))
//   MD_MWER = sum_g sum_i softmax(c_g)_i (e_i - sum_g e / n_g) + w * MD
//   MD_MWED = sum_g sum_i E_i (log E_i - log Q_i) + w * MD,           (kl_div(reduction="sum"))
//             E = softmax(e_g), Q = softmax(c_g / T_g), T_g = sum c_g / sum e_g (T depends
//             on s: its gradient is carried, as torch autograd does)
//   MD alone has weight 1; w = md_loss_weight.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/rescore.h"

// Dropout of BERT's train mode (modeling_bert.py: BertEmbeddings.dropout after the LayerNorm,
// the attention-probability dropout, BertSelfOutput / BertOutput dropout on the dense output
// before the residual add), inverted scaling x * 1/(1-p) on kept elements.  The keep bit of
// element e of site `site` in dropout step `step` is a counter-based draw,
//   keep = Philox4x32-10(counter = (e_lo, e_hi, site, step_hi), key = (seed, step_lo)).word0 >= thresh,
//   thresh = p * 2^32,
// with the 64-bit dropout step split into its words (the CLI keys epoch k's steps from k << 32, so
// every epoch has 2^32 steps of its own; steps below 2^32 have step_hi = 0, the round-3 masks),
// so no mask is stored: the backward recomputes the same bits, and a step is bitwise
// reproducible.  Sites: 0 = embeddings; layer l: 1 + 3l attention probabilities (element =
// its index in the saved-P layout), 2 + 3l self-output, 3 + 3l output (element = row * H + c).
// thresh == 0: off (p = 0, the fixture-pinned mode).
struct TrDrop {
    uint32_t seed = 0, step = 0, site = 0, thresh = 0, step_hi = 0;
    float scale = 1.f;
};

__host__ __device__ inline uint32_t tr_philox_w0(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                                 uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0, h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
        c0 = h1 ^ c1 ^ k0;
        c1 = l1;
        c2 = h0 ^ c3 ^ k1;
        c3 = l0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c0;
}

__host__ __device__ inline bool tr_keep(const TrDrop& d, unsigned long long e) {
    return tr_philox_w0((uint32_t)e, (uint32_t)(e >> 32), d.site, d.step_hi, d.seed, d.step) >= d.thresh;
}

__host__ __device__ inline float tr_drop(const TrDrop& d, unsigned long long e, float x) {
    if (d.thresh == 0) return x;
    return tr_keep(d, e) ? x * d.scale : 0.f;
}

// dst[e] = drop(src[e]) over n elements (dst may alias src)
hipError_t tr_dropout(float* dst, const float* src, long long n, const TrDrop& d, hipStream_t s);
// keep[e] = the keep bit of element e (test / export entry, rs_dropout_keep)
hipError_t tr_dropout_keep(uint8_t* keep, long long n, const TrDrop& d, hipStream_t s);

// h0 = drop(LN(x0)) (site 0); x0 and its statistics saved pre-dropout
hipError_t tr_embed_ln(const int* row_tok, const int* row_pos, int M, int vocab, const float* word,
                       const float* pos, const float* type0, const float* g, const float* b, float eps, int H,
                       float* x0, float2* st, float* h0, hipStream_t s, const TrDrop& d = TrDrop());
// y <- drop(y + bias) + res (saved), h = LN(y); bias == nullptr: plain LN of y (no dropout)
hipError_t tr_bias_res_ln(float* y, const float* bias, const float* res, int M, const float* g, const float* b,
                          float eps, int H, float2* st, float* h, hipStream_t s, const TrDrop& d = TrDrop());
hipError_t tr_bias_gelu(float* pre, const float* bias, float* act, int M, int N, hipStream_t s);
hipError_t tr_gelu_bwd(float* d, const float* pre, long long n, hipStream_t s);
hipError_t tr_bias(float* y, const float* bias, int M, int N, hipStream_t s);
// klen (nullable): sequence s attends to its first klen[s] tokens only (padded-batch rows)
// P saved before dropout; ctx = drop(P) V
hipError_t tr_attn_fwd(const float* qkv, const int* seq_off, const int* klen, const long long* pofs, int S,
                       int tmax, int H, int heads, float* P, float* ctx, hipStream_t s, const TrDrop& d = TrDrop());
hipError_t tr_attn_bwd(const float* qkv, const float* P, const float* dctx, const int* seq_off, const long long* pofs,
                       int S, int tmax, int H, int heads, float* dqkv, hipStream_t s, const TrDrop& d = TrDrop());
hipError_t tr_ln_bwd(const float* dy, const float* x, const float2* st, const float* g, float* dx, int M, int H,
                     hipStream_t s);
size_t tr_colsum_scratch(int M, int N);
hipError_t tr_colsum(const float* dy, const float* x, const float2* st, int M, int N, int mode, float* part,
                     float* out, int accumulate, hipStream_t s);
hipError_t tr_colsum_ln(const float* dy, const float* x, const float2* st, int M, int N, float* part, float* out_g,
                        float* out_b, hipStream_t s);
hipError_t tr_word_grad(const float* dx0, const int* utok, const int* toff, const int* rows, int n_uniq, int H,
                        float* dword, hipStream_t s);
hipError_t tr_pos_grad(const float* dx0, const int* seq_off, int S, int tmax, int H, float* dpos, hipStream_t s);
hipError_t tr_cls_fwd(const float* h, const int* seq_off, int S, int H, const float* w, const float* b, float* out,
                      hipStream_t s);
hipError_t tr_cls_bwd(const float* dsc, const float* h, const int* seq_off, int S, int H, const float* w, float* dh,
                      float* dw, float* db, hipStream_t s);
hipError_t tr_loss(const float* sc, const float* tgt, const float* am, const float* err, const int* utt_off,
                   int n_utt, int n_hyp, int kind, float md_w, float* dsc, float* uloss, float* loss, hipStream_t s);
hipError_t tr_ce(float* logits, const int* labels, int M, int V, float* row_loss, float* loss, hipStream_t s);
hipError_t tr_adamw(float* p, const float* g, float* m, float* v, long long n, float decay, float b1w, float b2,
                    float b2w, float step_size, float bc2_sqrt, float eps, hipStream_t s);
// fp32 GEMM on the f32-input MFMA (k_sgemm.hip): C[M][N] = A·B (+ C when accum), A read as
// [M][lda] with k contiguous (a_kc) or [K][lda] with rows contiguous, B as [N][ldb] (b_kc)
// or [K][ldb].  Few output tiles are split over K through ws (tr_sgemm_ws_floats floats),
// summed in split order: deterministic.
size_t tr_sgemm_ws_floats(int M, int N, int K);
int tr_sgemm_failed();      // a stream-K hand-off timed out since the last call (synchronous check)
hipError_t tr_sgemm(int M, int N, int K, const float* A, int lda, bool a_kc, const float* B, int ldb, bool b_kc,
                    float* C, int ldc, int accum, float* ws, size_t ws_floats, hipStream_t s);
