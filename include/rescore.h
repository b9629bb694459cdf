/*
 * librescore — C ABI of the MI355X-native N-best LM rescorer (gfx950 HIP kernels).
 *
 * The reference (ishine/ASR-Rescoring) is pure Python with no FFI; its seams on the hot
 * path are Python calls.  Each entry point below names the reference interface it
 * replaces (file:line, relative to the reference repo).  The Python host mirror in
 * asr-rescoring_amd/ binds these with ctypes (see INTEGRATION.md for the binding a
 * maintainer would add to the reference).
 *
 * Conventions
 *   - d_* pointers are device memory owned by the caller (e.g. the PyTorch caching
 *     allocator); h_* pointers are host memory read during the call only.
 *   - stream is a hipStream_t (torch.cuda.current_stream().cuda_stream); every call is
 *     asynchronous on it unless stated (the scoring calls synchronise at their end: range
 *     guard below).  No C++ exception crosses the ABI.
 *   - return 0 on success, a negative RS_E* code on failure; rs_last_error() gives a
 *     thread-local message.
 *   - A model handle is bound to one device and must not be used by two host threads
 *     at once.  Calls on one handle are ORDERED even across streams: they share the handle's
 *     workspace, LayerNorm gang-ticket words and flags, so a call issued on a different stream
 *     than the previous call first makes its stream wait (device-side) for the previous call's
 *     work.  Results are deterministic (no float atomics, fixed reduction orders).
 *   - The fused residual + LayerNorm GEMM (fp16x3 mode) exchanges row statistics between the
 *     N_pad / 256 workgroups of a row panel inside one launch (a gang).  Gangs are formed only
 *     from workgroups that have started, and the row panels come in lists that a gang takes from a
 *     counter, so the lists of gangs that never formed (workgroups held off by another tenant) are
 *     computed by those that did: the launch completes on whatever CUs it gets, with 3 free
 *     workgroup slots anywhere on the GPU for bert-base.  The hardware dispatches a grid's
 *     workgroups round-robin over the 32 shader engines (8 XCDs x 4); while another tenant fills a
 *     whole engine, the workgroups dispatched to it (of this kernel or any other) wait for it.
 *     Every wait inside a launch is bounded (statistics 1 s, gang formation 10 s): one that runs
 *     out ends the call in RS_EHIP instead of hanging.
 */
#ifndef RESCORE_H_
#define RESCORE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RS_OK 0
#define RS_EARG (-1)      /* bad argument / shape */
#define RS_EHIP (-2)      /* HIP runtime error */
#define RS_ESTATE (-3)    /* call order (e.g. scoring before rs_model_finalize) */
#define RS_ENOMEM (-4)
#define RS_EUNSUP (-5)    /* shape outside what the kernels support */

#define RS_DT_F32 0

#define RS_HEAD_MLM 1     /* BertForMaskedLM head: cls.predictions.* (MLM_PLL) */
#define RS_HEAD_CLS 2     /* RescoreBert head: linear.weight [1,H], linear.bias [1] */
#define RS_HEAD_EMB 4     /* encoder only: token embeddings (BERTScore, bert_score.utils.bert_encode) */

#define RS_LOSS_MD 0      /* RescoreBert training methods (RescoreBert/main.py:104-147) */
#define RS_LOSS_MWER 1    /* MD_MWER: MWER + md_loss_weight * MD */
#define RS_LOSS_MWED 2    /* MD_MWED: MWED + md_loss_weight * MD */

#define RS_BS_P 0         /* BERTScore component used as the MBR utility */
#define RS_BS_R 1
#define RS_BS_F 2

#define RS_FUSE_NORM 0    /* (1-w)*am/len + w*lm/len      rescore.py:51 */
#define RS_FUSE_LEGACY 1  /* (1-w)*am + w*lm              rescore_result/MLM_PLL/rescore.log:28 */
#define RS_FUSE_AM_NORM 2 /* (1-w)*am/len + w*lm          rescore_result/RMBR/BertScore/rescore_mbr_normalize.log:29 */

typedef struct rs_model rs_model;

/* transformers.BertConfig fields used by the reference (bert-base-chinese:
 * 21128/768/12/12/3072/512/2, eps 1e-12, [MASK] = 103). */
typedef struct rs_bert_cfg {
    int32_t vocab, hidden, layers, heads, intermediate, max_pos, type_vocab;
    float ln_eps;
    int32_t mask_id;
    int32_t heads_mask;   /* RS_HEAD_MLM | RS_HEAD_CLS */
    int32_t precision;    /* RS_PREC_FP16 or RS_PREC_FP16X3 */
} rs_bert_cfg;

/* GEMM operand precision.  FP16X3 (the default of every scorer): each fp32 operand x is
 * split into fp16 hi + lo (lo scaled by 64) and the three significant products
 * A_hi.W_hi + A_hi.W_lo + A_lo.W_hi are accumulated in fp32 on the fp16 MFMA — by the
 * split-operand kernel from two-part images, the third product's factors formed in registers
 * (fp32-level accuracy: PLL ~1e-7 relative of the fp32 reference, 3 MFMA products per
 * algorithmic one).  FP16: fp16 MFMA inputs, fp32 accumulation (opt-in reduced-precision
 * mode: per-row log-probs within ~1e-4 relative).  Both modes hold operands in fp16 images,
 * so |x| <= 65504: weights beyond it fail rs_model_finalize, activations beyond it make the
 * scoring call fail with RS_EUNSUP (range guard, below). */
#define RS_PREC_FP16 0
#define RS_PREC_FP16X3 1

int rs_version(void);
const char* rs_last_error(void);

/* Replaces BertForMaskedLM.from_pretrained / RescoreBert(...) construction
 * (MLM_PLL/main.py:184, RescoreBert/model.py:5-11).  Requires hidden % 256 == 0,
 * head_dim == 64, intermediate % 128 == 0. */
int rs_model_create(const rs_bert_cfg* cfg, int device, rs_model** out);

/* Replaces model.load_state_dict(torch.load(checkpoint)) (MLM_PLL/main.py:185-186,
 * RescoreBert/main.py:250-251): one HF state_dict tensor by key, host fp32. */
int rs_model_set_tensor(rs_model* m, const char* hf_key, const void* host_ptr, int dtype,
                        const int64_t* shape, int ndim);

/* Packs the tensors into the kernel layouts (fp16 GEMM weights, fused QKV) on device.
 * Fails with RS_ESTATE naming the first missing key, RS_EUNSUP for a weight outside the fp16 range.
 * fp16x3: the split-operand GEMMs form 64 W_hi in fp16, so a model with a projection weight of
 * |w| >= 1023.75 is packed without them and runs the K-concatenated fp16x3 form (same accuracy,
 * slower); scores are never affected. */
int rs_model_finalize(rs_model* m);

/* Sizes the activation workspace for up to max_rows token rows per launch chunk
 * (>= 512).  Optional: scoring calls reserve a default on first use. */
int rs_model_reserve(rs_model* m, int64_t max_rows);

/* Range guard of the scoring calls (rs_pll_score, rs_masked_logprob, rs_cls_score,
 * rs_token_embed, rs_bertscore_recall): after the last launch the call checks its outputs
 * for non-finite values (an operand image that overflowed fp16 turns every dependent score
 * into inf / NaN), synchronises `stream` and returns RS_EUNSUP with a message instead of
 * handing back non-finite scores.  These calls therefore return with their work complete.
 * The same report carries RS_EHIP when a fused residual-LayerNorm GEMM timed out waiting for
 * its row statistics (each call reports only its own).
 *
 * rs_model_set_sync_check(m, 0) defers that report: the calls only enqueue the check (they stay
 * asynchronous on `stream`), the flags accumulate on the device, and rs_check(m, stream)
 * synchronises `stream`, reports (RS_EUNSUP / RS_EHIP) and clears them.  on = 1 restores the
 * default; call rs_check first so nothing pending is dropped.  In deferred mode a statistics-wait
 * timeout (RS_EHIP) is sticky on the device until rs_check: every fused-LayerNorm launch after it
 * drains at once (fail-fast: no further waits), so EVERY result produced between the timeout and
 * the rs_check that reports it is invalid and must be discarded — not only the timed-out call's.  No reference counterpart (the
 * reference's forward is synchronous PyTorch-CPU, MLM_PLL/main.py:83-107). */
int rs_model_set_sync_check(rs_model* m, int on);
int rs_check(rs_model* m, void* stream);

/* MLM_PLL scoring (MLM_PLL/preprocess.py:9-30 + MLM_PLL/main.py:83-107):
 *   d_tok      int32 [h_hyp_off[n_hyp]]  hypotheses as [CLS] w_1..w_L [SEP]
 *   h_hyp_off  int32 [n_hyp + 1]         host offsets into d_tok (T_h = L_h + 2 >= 3)
 *   d_pll      float64 [n_hyp]           sum_p log p(w_p | w_{\p}) accumulated in row
 *                                        order p = 1..L (== output_score[u][h])
 *   d_row_lp   float32 [sum_h L_h] or NULL: per masked row log-prob (== token_score)
 * The L masked copies are expanded on device. */
int rs_pll_score(rs_model* m, const int32_t* d_tok, const int32_t* h_hyp_off, int32_t n_hyp,
                 double* d_pll, float* d_row_lp, void* stream);

/* Row-level MLM drop-in (MLM_PLL/main.py:89-105 for an arbitrary batch):
 *   d_ids      int32 ragged sequences (already masked), h_seq_off int32 [n_seq+1] host
 *   h_query    int32 [n_seq] host   position of the masked token in each sequence
 *   d_label    int32 [n_seq]        label id at that position
 *   d_out      float32 [n_seq]      log_softmax(logits[query])[label] */
int rs_masked_logprob(rs_model* m, const int32_t* d_ids, const int32_t* h_seq_off,
                      const int32_t* h_query, const int32_t* d_label, int32_t n_seq,
                      float* d_out, void* stream);

/* RescoreBert scoring (RescoreBert/model.py:13-21, RescoreBert/main.py:156-158):
 * CLS hidden of the last layer -> Linear(H, 1).  d_out float32 [n_hyp]. */
int rs_cls_score(rs_model* m, const int32_t* d_tok, const int32_t* h_hyp_off, int32_t n_hyp,
                 float* d_out, void* stream);

/* Per-kernel-kind device timing (HIP events around every launch of that kind, on the
 * call's stream).  Enable before a scoring call; read after it (synchronises).
 * kind: RS_K_QKV, RS_K_OPROJ, RS_K_FFN1, RS_K_FFN2, RS_K_DECODER, RS_K_ATTN, RS_K_OTHER.
 * flops = algorithmic FLOPs of the launches of that kind (2*M*N*K over valid rows). */
#define RS_K_QKV 0
#define RS_K_OPROJ 1
#define RS_K_FFN1 2
#define RS_K_FFN2 3
#define RS_K_DECODER 4
#define RS_K_ATTN 5
#define RS_K_OTHER 6
#define RS_K_COUNT 7
int rs_profile_enable(rs_model* m, int on);
int rs_profile_read(rs_model* m, int kind, double* ms, int64_t* launches, double* flops);

void rs_model_destroy(rs_model* m);

/* RMBR CER utility (RMBR/utility_functions.py:28-33 via RMBR/mbr.py:5-28): the
 * pairwise Levenshtein matrix of every utterance's hypotheses, computed once.
 *   d_chars   int32 symbols, d_str_off int32 [n_str+1], d_utt_off int32 [n_utt+1]
 *             (strings of utterance u = utt_off[u]..utt_off[u+1])
 *   d_mat_off int64 [n_utt+1] offsets of each n_u x n_u block in d_ed (row-major)
 *   d_ed      int32 out: d_ed[mat_off[u] + i*n_u + j] = ed(string_i, string_j)
 * Myers/Hyyro bit-parallel: one 64-bit word when the shorter string of a pair has <= 64
 * symbols, 64-row words with carried horizontal deltas beyond; exact when the shorter
 * string has <= 16384 symbols, -1 otherwise (the Python wrappers reject such inputs). */
int rs_pairwise_edit(const int32_t* d_chars, const int32_t* d_str_off, const int32_t* d_utt_off,
                     const int64_t* d_mat_off, int32_t n_utt, int32_t max_n, int32_t* d_ed,
                     void* stream);

/* Token embeddings of the BERTScore utility (RMBR/utility_functions.py:9-22 ->
 * bert_score.utils.get_bert_embedding / bert_encode with the model truncated to cfg.layers
 * layers — bert_score uses 8 for bert-base-chinese — and greedy_cos_idf's per-token L2
 * normalisation), row = token position in d_tok (h_hyp_off: host int32 [n_hyp+1], hypotheses
 * as [CLS] w.. [SEP]).  d_emb layout by the model's precision: RS_PREC_FP16X3 — the two-part
 * image fp16 [hyp_off[n_hyp], 2*hidden], row = [hi | lo*64], e = hi + lo/64 (fp32-class, ~22
 * bits); RS_PREC_FP16 — fp16 [hyp_off[n_hyp], hidden]. */
int rs_token_embed(rs_model* m, const int32_t* d_tok, const int32_t* h_hyp_off, int32_t n_hyp,
                   void* d_emb, void* stream);

/* bert_score.score(cands=[hyp_i], refs=[hyp_j], idf=False) for every ordered pair of each
 * utterance's hypotheses, as the recall matrix
 *   d_rmat[mat_off(u) + i*n_u + j] = R(cand = hyp_i, ref = hyp_j),
 *   mat_off(u) = sum_{v<u} n_v^2 (n_u = h_utt_off[u+1] - h_utt_off[u]);
 * P(i|j) = R(j|i), F = 2PR/(P+R).  R = mean over ref j's tokens except [CLS]/[SEP] of the max
 * cosine over all of cand i's tokens; 0 when either hypothesis is empty (T == 2).  Cosines:
 * RS_PREC_FP16X3 three fp16 products of the two-part embeddings, fp32 accumulation (fp32-class);
 * RS_PREC_FP16 one.
 * d_rmat0 (optional, same layout): each maximum taken as max(m, 0) — bert_score's value when
 * the cand is shorter than the longest cand of its pair batch (the padded positions' masked
 * cosine 0 joins the max, bert_score/utils.py greedy_cos_idf); the caller picks R or R0 per
 * pair from its batch layout (bertscore.py).
 * h_hyp_off[0] == 0, h_utt_off[0] == 0 (host arrays); every hypothesis has T >= 2. */
int rs_bertscore_recall(rs_model* m, const int32_t* d_tok, const int32_t* h_hyp_off,
                        const int32_t* h_utt_off, int32_t n_utt, float* d_rmat, float* d_rmat0, void* stream);

/* RMBR mbr_decode (RMBR/mbr.py:5-28) with the BERTScore utility component `which`
 * (RS_BS_P/R/F) of cand hyp_i against ref hyp_j, from the rs_bertscore_recall matrix;
 * summation and argmax as rs_mbr_scores. */
int rs_mbr_scores_bs(const float* d_rmat, const int64_t* d_mat_off, const int32_t* d_utt_off, int32_t n_utt,
                     int32_t k, int32_t which, float* d_scores, int32_t* d_argmax, void* stream);

/* ---- Levenshtein alignment with backtrace (espnet_data/preprocess/align.py:5-97
 * levenshtein_distance_alignment) -----------------------------------------
 * Pair p aligns ref tokens d_ref[d_ref_off[p] .. d_ref_off[p+1]) with hyp tokens
 * d_hyp[d_hyp_off[p] .. ) (int32 token ids, any values; 0 <= length <= 4096, max_len = the
 * longest list of the call).  Reference rules: rows = hyp, columns = ref, both with a start
 * sentinel; equal tokens take the diagonal cost as "U"; otherwise S = diag + 1, replaced only
 * by a strictly smaller I = left + 1, then by a strictly smaller D = up + 1; first column D,
 * first row I; traceback from the end: U / S consume both, D = hyp-only token (ref "*"),
 * I = ref-only token (hyp "*"); output in forward order (the reference reverses its lists).
 * Outputs at d_out_off[p] (int64, room for len(ref) + len(hyp) entries): d_ops int8
 * (RS_AL_U / _S / _I / _D), d_ref_idx / d_hyp_idx int32 (index into the pair's ref / hyp
 * tokens, -1 = "*"), d_n[p] = the alignment's length.  d_lab: uint8 scratch of
 * (len(hyp) + 1) * (len(ref) + 1) bytes per pair at d_lab_off[p] (int64).  Async on `stream`. */
#define RS_AL_U 0
#define RS_AL_S 1
#define RS_AL_I 2
#define RS_AL_D 3
int rs_align(const int32_t* d_ref, const int32_t* d_ref_off, const int32_t* d_hyp, const int32_t* d_hyp_off,
             int32_t n_pairs, const int64_t* d_lab_off, uint8_t* d_lab, const int64_t* d_out_off, int8_t* d_ops,
             int32_t* d_ref_idx, int32_t* d_hyp_idx, int32_t* d_n, int32_t max_len, void* stream);

/* ---- RescoreBert training (RescoreBert/main.py:82-229) ---------------------------------
 * A trainer holds fp32 parameters (HF keys as for rs_model; bert.pooler.* is accepted and
 * ignored — RescoreBert's loss never reaches it), their gradients and AdamW moments.
 * rs_train_step_cls runs forward (activations kept), the distillation loss, the full
 * backward and (opts->update) one torch.optim.AdamW step.  Losses (RescoreBert/main.py:104-147;
 * train.h), over utterance groups g given by h_utt_off (the reference's reshape(-1, n_best)):
 *   MD      = sum_i (s_i - t_i)^2                            (MSELoss(reduction="sum"))
 *   MD_MWER = sum_g sum_i softmax(c_g)_i (cer_i - mean_g cer) + md_loss_weight * MD
 *   MD_MWED = sum_g KL(softmax(cer_g) || softmax(c_g / T_g)) + md_loss_weight * MD,
 *             T_g = sum c_g / sum cer_g (differentiated through), c = s + am.
 * Dropout (BERT train mode; the reference trains under model.train(), p = 0.1 by default):
 * hidden_dropout after the embedding LayerNorm and on the BertSelfOutput / BertOutput dense
 * outputs, attn_dropout on the attention probabilities, inverted scaling, on steps with
 * update >= 0 (the dev-loss pass, update = -1, is eval mode).  The keep bits are
 * counter-based (Philox4x32-10 keyed by dropout_seed and the trainer's dropout-step counter,
 * rs_trainer_dropout_step), so a step is bitwise reproducible; torch's RNG stream cannot be
 * matched, and the fixture-pinned runs use p = 0. */
typedef struct rs_trainer rs_trainer;
typedef struct rs_train_opts {
    int32_t loss;          /* RS_LOSS_MD / RS_LOSS_MWER / RS_LOSS_MWED */
    float md_loss_weight;  /* weight of MD in MD_MWER / MD_MWED (MD alone has weight 1) */
    float lr, beta1, beta2, eps, weight_decay;   /* torch.optim.AdamW arguments */
    int32_t update;        /* 1: backward + AdamW step; 0: backward only (gradients kept);
                              -1: forward + loss only (the reference's dev-loss pass) */
    float hidden_dropout;  /* BertConfig.hidden_dropout_prob (0 = off) */
    float attn_dropout;    /* BertConfig.attention_probs_dropout_prob (0 = off) */
    uint32_t dropout_seed;
} rs_train_opts;

/* cfg->heads_mask: RS_HEAD_CLS (RescoreBert) or RS_HEAD_MLM (MLM fine-tuning); shapes as
 * rs_model_create (T <= 128 per sequence). */
int rs_trainer_create(const rs_bert_cfg* cfg, int device, rs_trainer** out);
int rs_trainer_set_tensor(rs_trainer* t, const char* hf_key, const void* host_ptr, int dtype,
                          const int64_t* shape, int ndim);
int rs_trainer_finalize(rs_trainer* t);
/* d_tok/h_hyp_off as rs_cls_score; h_utt_off int32 [n_utt+1] groups hypotheses by utterance;
 * d_target (mlm_pll_score), d_am (hyps_am_score), d_err (hyps_cer) float32 [n_hyp] (am/err
 * only for MWER/MWED);
 * d_scores (nullable) float32 [n_hyp] out; d_loss float32 [1] out.  Synchronises `stream`. */
int rs_train_step_cls(rs_trainer* t, const int32_t* d_tok, const int32_t* h_hyp_off, int32_t n_hyp,
                      const int32_t* h_utt_off, int32_t n_utt, const float* d_target, const float* d_am,
                      const float* d_err, const rs_train_opts* opts, float* d_scores, float* d_loss,
                      void* stream);
/* MLM fine-tuning step (MLM_PLL/main.py:73-161 run_one_epoch / mlm_finetune_bert; trainer
 * created with heads_mask RS_HEAD_MLM — cls.predictions.* with the decoder tied to the word
 * embeddings): d_ids / d_labels int32 rows (h_seq_off host int32 [n_seq+1]).  h_key_len (host
 * int32 [n_seq], nullable = whole rows): row s attends to its first h_key_len[s] tokens only —
 * the reference's padded batch (collate MLM_PLL/main.py:28-54: ids / labels padded with 0,
 * attention_mask 0) is rows of the batch's longest length whose pad positions are queries but
 * not keys.  loss = mean over ALL positions of the rows (pads included, label 0) of the CE of
 * BertForMaskedLM's logits (modeling_bert CrossEntropyLoss, MLM_PLL/main.py:89-97).
 * Synchronises `stream`. */
int rs_train_step_mlm(rs_trainer* t, const int32_t* d_ids, const int32_t* h_seq_off, int32_t n_seq,
                      const int32_t* h_key_len, const int32_t* d_labels, const rs_train_opts* opts,
                      float* d_loss, void* stream);
/* The dropout-step counter: the key the next dropout-active step uses (then incremented). */
int64_t rs_trainer_dropout_step(const rs_trainer* t);
/* Sets it (0 .. 2^63-1; a 64-bit counter whose high word is a Philox counter word and low word
 * the second key word): part of the resume state — the CLI starts epoch k at k << 32, so every
 * epoch has 2^32 dropout steps of its own and a run resumed at epoch k draws the masks of the
 * straight run. */
int rs_trainer_set_dropout_step(rs_trainer* t, int64_t step);
/* d_keep uint8 [n]: the keep bit the trainer's kernels use for element e of dropout site
 * `site` (0 = embeddings; layer l: 1 + 3l attention probabilities in the saved-P layout,
 * 2 + 3l self-output, 3 + 3l output, element = row * hidden + column) in dropout step `step`
 * with probability p.  Test / export entry (masks fed to the CPU oracle). */
int rs_dropout_keep(uint32_t seed, uint64_t step, uint32_t site, float p, int64_t n, uint8_t* d_keep, void* stream);
/* Synchronous copies of one parameter / its last gradient (numel must match). */
int rs_trainer_get_tensor(rs_trainer* t, const char* hf_key, void* host_out, int64_t numel);
int rs_trainer_get_grad(rs_trainer* t, const char* hf_key, void* host_out, int64_t numel);
/* A fresh AdamW state (moments and step count zeroed; MLM_PLL/main.py:76 builds its
 * optimizer inside every epoch). */
int rs_trainer_reset_optimizer(rs_trainer* t);
void rs_trainer_destroy(rs_trainer* t);

/* RMBR mbr_decode scores for top-k (RMBR/mbr.py:17-22):
 *   score[u][i] = float32 torch-CPU-order sum over j != i (j < k) of
 *                 float32(1 - ed(hyp_j, hyp_i) / len(hyp_j));  argmax[u] = first max.
 * d_len int32 [n_str]; d_scores float32 [n_utt * k]; d_argmax int32 [n_utt]. */
int rs_mbr_scores(const int32_t* d_ed, const int64_t* d_mat_off, const int32_t* d_utt_off,
                  const int32_t* d_len, int32_t n_utt, int32_t k, float* d_scores,
                  int32_t* d_argmax, void* stream);

/* Fusion + argmax over a weight grid (rescore.py:37-58), fp64 with the reference's
 * operation order, no contraction.  Utterance u has hypotheses utt_off[u]..utt_off[u+1]
 * (first n_best of them used).  d_argmax int32 [n_w * n_utt] (first max). */
int rs_fuse_rerank(const double* d_am, const double* d_lm, const int32_t* d_len,
                   const int32_t* d_utt_off, int32_t n_utt, int32_t n_best, const double* d_w,
                   int32_t n_w, int32_t mode, int32_t* d_argmax, void* stream);

/* Corpus-CER numerators for every weight (jiwer.cer at rescore.py:40): edits[w] =
 * sum_u ed_ref[utt_off[u] + argmax[w][u]] over d_ed_ref int32 [n_hyp] (edit distance of
 * each hypothesis to its reference).  d_edits int64 [n_w]. */
int rs_corpus_edits(const int32_t* d_ed_ref, const int32_t* d_utt_off, const int32_t* d_argmax,
                    int32_t n_utt, int32_t n_w, int64_t* d_edits, void* stream);

/* Edit distance of every hypothesis to its utterance's reference (the per-hypothesis
 * table behind jiwer.cer's numerator): d_ref_chars/d_ref_off int32 [n_utt+1] are the
 * references, hypotheses as in rs_pairwise_edit (any number per utterance; the same length
 * limit).  d_ed_ref int32 [n_hyp]. */
int rs_ref_edit(const int32_t* d_chars, const int32_t* d_str_off, const int32_t* d_utt_off,
                const int32_t* d_ref_chars, const int32_t* d_ref_off, int32_t n_utt,
                int32_t* d_ed_ref, void* stream);

/* ---- Native host front end (host-only, no GPU) ------------------------
 * Replaces the tokenizer calls of MLM_PLL/preprocess.py:9-30 (BertTokenizer.tokenize +
 * convert_tokens_to_ids per hypothesis text) and RescoreBert/preprocess.py:8-55, and the
 * score writer util/saving.py:14-16. */

/* Load a BERT vocab.txt (one token per line, id = line index, later duplicates win).
 * Returns an opaque handle or NULL (rs_last_error-style message not set: path unreadable). */
void* rs_vocab_load(const char* path);
int rs_vocab_size(const void* vocab);
void rs_vocab_free(void* vocab);

/* BertTokenizer(vocab, do_lower_case=True).tokenize + convert_tokens_to_ids for n NFC UTF-8
 * texts, optionally wrapped in [CLS] .. [SEP] (add_special != 0): the ragged token layout
 * rs_pll_score / rs_cls_score consume.  ids int32 [cap], off int64 [n+1].  Returns the total
 * id count (> cap: only the first cap ids were written; call again with a larger buffer),
 * or < 0 on bad arguments. */
int64_t rs_tokenize_batch(const void* vocab, const char* const* texts, int32_t n, int32_t add_special,
                          int32_t* ids, int64_t cap, int64_t* off);

/* {utt_id: {hyp_id: score}} written byte-identical to json.dump(obj, f, indent=4,
 * ensure_ascii=False) (util/saving.py:14-16); hyp_off int32 [n_utt+1] indexes hyp_ids and
 * scores (float64, Python repr formatting).  Returns 0 or -1 (file not writable). */
int rs_json_write_scores(const char* path, int32_t n_utt, const char* const* utt_ids,
                         const int32_t* hyp_off, const char* const* hyp_ids, const double* scores);

#ifdef __cplusplus
}
#endif
#endif /* RESCORE_H_ */
