// Shared definitions for the gfx950 kernels and the C-ABI host code.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef _Float16 f16;
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define RS_WAVE 64

// GEMM epilogues (C = A[M,K] . W[N,K]^T, fp32 accumulate):
enum EpiKind {
    EPI_BIAS_F16 = 0,   // out16 = acc + bias                      (fused QKV projection)
    EPI_GELU_F16 = 1,   // out16 = gelu(acc + bias)                (BertIntermediate)
    EPI_GELU_F32 = 2,   // out32 = gelu(acc + bias)                (MLM transform, pre-LN)
    EPI_RES_F32 = 3,    // out32 = acc + bias + res32              (BertSelfOutput / BertOutput, pre-LN)
    EPI_LSE = 4,        // per-row partial (max, sum exp) over a 64-column slab + label logit
    EPI_BIAS_F32 = 5,   // out32 = acc + bias                      (QKV in the fp16x3 precision mode)
    EPI_RESLN_F32 = 6,  // out32 = acc + bias + LN(res32)          (same, residual kept pre-LN:
                        //   LN rebuilt from res_stats/res_g/res_b; out may alias res)
    EPI_LNRES_IMG = 7,  // h <- image(LN(acc + bias + h)), h the two-part image in out, in place
                        //   (split-operand residual blocks; row statistics exchanged between the
                        //   column tiles of a row panel inside the launch: gemm_x3s_kernel)
};

struct EpiArgs {
    const float* bias;     // [N]
    const float* res;      // [M, ldc] fp32 residual (EPI_RES_F32; pre-LN sum for EPI_RESLN_F32)
    const float2* res_stats;  // [M] (mean, 1/sqrt(var + eps)) of res rows (EPI_RESLN_F32)
    const float* res_g;    // [N] LayerNorm weight / bias applied to res (EPI_RESLN_F32)
    const float* res_b;
    void* out;             // [M, ldc]
    int ldc;
    int m_valid;           // rows >= m_valid are not stored
    int n_valid;           // columns >= n_valid are masked (EPI_LSE vocab padding)
    float2* lse_part;      // [M, n_parts] (max, sum exp) (EPI_LSE)
    int n_parts;
    const int* label;      // [M] label column per row (EPI_LSE)
    float* label_logit;    // [M]
    int kx;                // fp16 operand image width factor of the output (EPI_GELU_F16): 1 or 3
    int nlog;              // logical N (column offset of the image sections)
    int group_m;           // tile order: row panels per group (set by launch_gemm)
    // EPI_RESLN_F32 with res_o16 != null (deferred BertSelfOutput residual): the residual is
    // LN(LN0(res) + o16) with LN0 = (res_stats0, res_g0, res_b0) and LN = (res_stats, res_g,
    // res_b), i.e. the post-attention stream ln_res_rows did not write back (WX = false)
    const f16* res_o16;    // [M, ldc] fp16 O-projection output (bias included)
    const float2* res_stats0;
    const float* res_g0;
    const float* res_b0;
    // EPI_LNRES_IMG: LN = (res_g, res_b, ln_eps) over nlog columns; lnx: lnres_granules(M)
    // 8-B granules [M/256][N/256][256][2] {ln_tag, sum | M2}, then [M/256] {ln_tag, panel list}
    // (zeroed once by the owner); lncnt:
    // lnres_counter_bytes() of gang-ticket words and gang-id slots (zeroed once by the owner, left
    // zeroed by every launch); lnerr (sticky, the caller's): set to 1 when a statistics or gang wait
    // timed out; ln_tag: set by the launch
    void* lnx;
    unsigned* lncnt;
    unsigned* lnerr;
    unsigned ln_tag;
    float ln_eps;
    int diag;              // EPI_LNRES_IMG: 8 = every wait times out (RS_LNFUSE_DIAG, tests); 0 in production
    unsigned long long* dbg;  // stamp builds only (rs_debug_stamps): per-workgroup phase cycle sums
};
// <= 4 column tiles of 256 rows x 2 statistics granules, then one list-claim granule per row panel
inline size_t lnres_granules(int m_pad) { return (size_t)m_pad * 4 * 2 + (size_t)m_pad / 256 + 1; }

// fp16 operand image of an fp32 activation row with logical width K:
//   kx == 1: [hi]                          (RS_PREC_FP16)
//   kx == 3: [hi | hi/64 | (x - hi)*64]    (RS_PREC_FP16X3, K-concatenated GEMM form)
//   kx == 2: hi and lo = (x - hi)*64 INTERLEAVED per 32-column K-step (RS_PREC_FP16X3,
//            split-operand GEMM form): [hi 0..31 | lo 0..31 | hi 32..63 | lo 32..63 | ...], so
//            one K-step of a row is one 128-B line and the x3s kernel's LDS-DMA requests whole
//            lines (round 6; the planar [hi | lo] form requested two 64-B halves per row and
//            K-step, and that kernel's K loop is request-rate bound: profiles/r5kline_*).
//            Column c's hi part sits at il_hi(c), its lo part 32 halves later.  The x3s kernel
//            forms 64 W_hi in registers; its weights are the same interleaved [W_hi | W_lo*64].
// paired with the weight image [W_hi | W_lo*64 | W_hi/64] the K-concatenated MFMA product is
// A_hi.W_hi + A_hi.W_lo + A_lo.W_hi (the power-of-two factors cancel exactly): fp32-level
// accuracy from fp16 MFMA in one accumulator.  The factors keep the lo parts out of the fp16
// subnormal range, which the f16 MFMA flushes: lo = x - hi is subnormal for |x| < 0.25, and
// weights of |W| ~ 0.05 have W_lo ~ 1e-5 (unscaled, those products were lost).
constexpr float X3_UP = 64.f, X3_DOWN = 1.f / 64.f;
__host__ __device__ __forceinline__ int il_hi(int c) { return ((c & ~31) << 1) | (c & 31); }
__device__ __forceinline__ f16 x3_mid(f16 hi) { return (f16)((float)hi * X3_DOWN); }
// lo = RNE(64 (v - hi)), formed as one fma of the fp16 hi with 64 v (v_fma_mix: 64 (v - hi) is
// exact in fp32, so the single rounding to fp16 gives the same bits as (v - hi) * 64 rounded)
__device__ __forceinline__ f16 x3_lo(float v, f16 hi) { return (f16)__builtin_fmaf((float)hi, -X3_UP, v * X3_UP); }
__device__ __forceinline__ void put_split(f16* row, int c, int K, int kx, float v) {
    const f16 hi = (f16)v;
    if (kx == 2) {
        row[il_hi(c)] = hi;
        row[il_hi(c) + 32] = x3_lo(v, hi);
        return;
    }
    row[c] = hi;
    if (kx == 3) {
        row[K + c] = x3_mid(hi);
        row[2 * K + c] = x3_lo(v, hi);
    }
}
// c % 4 == 0 (the four columns lie in one 32-column K-step)
__device__ __forceinline__ void put_split4(f16* row, int c, int K, int kx, float4 v) {
    const half4 hi = {(f16)v.x, (f16)v.y, (f16)v.z, (f16)v.w};
    const int ch = kx == 2 ? il_hi(c) : c;
    *(half4*)(row + ch) = hi;
    if (kx >= 2) {
        const half4 lo = {x3_lo(v.x, hi[0]), x3_lo(v.y, hi[1]), x3_lo(v.z, hi[2]), x3_lo(v.w, hi[3])};
        *(half4*)(row + (kx == 2 ? ch + 32 : 2 * K + c)) = lo;
    }
    if (kx == 3) {
        const half4 mid = {x3_mid(hi[0]), x3_mid(hi[1]), x3_mid(hi[2]), x3_mid(hi[3])};
        *(half4*)(row + K + c) = mid;
    }
}
// value of column c of a kx == 2 image row: hi + lo/64
__device__ __forceinline__ float2 il_parts(const f16* row, int c) {
    return make_float2((float)row[il_hi(c)], (float)row[il_hi(c) + 32]);
}

// Per-sequence metadata of a scoring call (structure of arrays, device).  A "sequence"
// is one BERT input: a masked copy of a hypothesis (MLM_PLL), a hypothesis
// (RescoreBert) or a caller-provided row (masked_logprob).
struct SeqMeta {
    const int* tok_off;    // offset of the sequence's [CLS] in the token buffer
    const int* len;        // T
    const int* mask_pos;   // position replaced by [MASK] on device, -1 = none
    const int* query;      // row whose last-layer state is scored
    const int* label;      // label id at query, -1 = take tokens[tok_off + query]
    const int* row;        // first token row of the sequence (global row index)
    const int* urow_h;     // layer-0 dedup: first unique row of the sequence's hypothesis (chunk-local)
    const int* urow_m;     // layer-0 dedup: the sequence's [MASK] unique row (chunk-local)
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

// ---- launchers (defined in k_gemm.hip / k_bert.hip / k_rerank.hip) ---------------------
// tag != 0: the same kernel instantiated under a distinct VAR tag bit (kernel name only), so
// rocprofv3 separates the O-projection (tag 1) and BertOutput (tag 2) launches from the QKV
// launches of the same epilogue
hipError_t launch_gemm(int epi, const f16* A, const f16* W, int M_pad, int N_pad, int K,
                       const EpiArgs& ep, hipStream_t st, int tag = 0);
// split-operand fp16x3 GEMM (gemm_x3s_kernel): A the interleaved two-part image [M_pad, 2K]
// (kx == 2 above), W rows of ldw >= 2K halfs starting with the interleaved [W_hi | W_lo*64] image
// (ldw = 2K: the packed split-operand weights); epi EPI_BIAS_F32, EPI_GELU_F16 (interleaved
// two-part image out) or EPI_LNRES_IMG.  N_pad % 256 == 0, K % 32 == 0, K >= 64.
hipError_t launch_gemm_x3s(int epi, const f16* A, const f16* W, int ldw, int M_pad, int N_pad, int K,
                           const EpiArgs& ep, hipStream_t st);
int gemm_row_align();   // M padding granularity required by launch_gemm
int gemm_lnres_workgroups(int N_pad);   // grid of the fused residual + LayerNorm GEMM (whole gangs)
size_t lnres_counter_bytes();           // EpiArgs.lncnt size

// kx: width factor of the fp16 operand images written (1 or 3, see put_split);
// qkv32: the QKV projection is fp32 (fp16x3 mode) instead of fp16.
// LayerNorm output of one element from its row statistics: the single expression every
// kernel uses, so an LN rebuilt downstream (EPI_RESLN_F32, attention_query) is bit-identical
// to the one the LN kernel writes.
// Every multiply-add of the LayerNorm is spelled out (fmaf / __fmul_rn): left to -ffp-contract,
// the same source contracted differently in different kernels (embed_ln vs embed_unique), and
// the rows two kernels must produce bit-identically (layer-0 dedup) differed in the last bit.
__device__ __forceinline__ float ln_apply(float x, float2 st, float g, float b) {
    return __builtin_fmaf(__fmul_rn(x - st.x, st.y), g, b);
}

// embed_ln writes the pre-LN embedding sum (x32), its row statistics and the fp16 operand
// image of LN(x); ln_rows writes the operand image, the statistics and (y32 != null) LN(x).
hipError_t launch_embed_ln(const int* tok, SeqMeta sm, int s0, int s1, int row0, int mask_id,
                           int vocab, const float* word, const float* pos, const float* type0,
                           const float* g, const float* b, float eps, int H, float* x32,
                           float2* stats, f16* h16, int kx, hipStream_t st);
hipError_t launch_ln_rows(const float* x, int rows, const float* g, const float* b, float eps,
                          int H, float* y32, float2* stats, f16* y16, int kx, hipStream_t st);
// x = LN(x32; stats, pg, pb) + o16, then stats_out / fp16 image of LN(x; g, b) (kx == 1);
// write_x: x written back into x32 (else x32 is left as is and the consumer rebuilds x from
// x32, stats, o16: EpiArgs.res_o16 or a second ln_res_rows).  o16b != null (needs write_x):
// two residual blocks, x = LN(LN(x32; stats, pg, pb) + o16; stats1, g1, b1) + o16b.
// stats_out may alias stats.
hipError_t launch_ln_res_rows(float* x32, const float2* stats, float2* stats_out, const float* pg, const float* pb,
                             const f16* o16, int rows, const float* g, const float* b, float eps, int H,
                             f16* y16, bool write_x, hipStream_t st, const float2* stats1 = nullptr,
                             const float* g1 = nullptr, const float* b1 = nullptr, const f16* o16b = nullptr);
// fp16x3 split-operand mode: x32 <- LN(x32; stats, pg, pb) + o32 (o32 = the projection's fp32
// output, bias included), then its statistics (stats_out, may alias stats) and the operand image
// of LN(x32; g, b) with width factor kx
hipError_t launch_ln_res32(float* x32, const float2* stats, float2* stats_out, const float* pg, const float* pb,
                           const float* o32, int rows, const float* g, const float* b, float eps, int H, f16* y16,
                           int kx, hipStream_t st);
hipError_t launch_ln_res_img(f16* h16, const float* o32, int rows, const float* g, const float* b, float eps, int H,
                             hipStream_t st);
// Unique layer-0 rows (dedup): for every hypothesis of the chunk its T rows, and every
// sequence's [MASK] row, as the fp16 operand image of LN(embedding) (rows of SeqMeta.urow_*)
hipError_t launch_embed_unique(const int* tok, SeqMeta sm, int s0, int s1, int mask_id, int vocab,
                               const float* word, const float* pos, const float* type0, const float* g,
                               const float* b, float eps, int H, f16* h16u, int kx, hipStream_t st);
// BERTScore recall matrix (k_bertscore.hip); items = (utterance, j0, j1, -) ref-column runs of
// at most bertscore_cols(two) columns; two: emb is the two-part image (split-operand cosines)
int bertscore_cols(bool two);
hipError_t launch_bertscore_recall(const f16* emb, int H, const int* hyp_off, const int* utt_off,
                                   const long long* mat_off, const int4* items, int n_items, float* rmat, float* rmat0,
                                   hipStream_t st, bool two = false);
// Last hidden state, L2-normalised per token, at out[(tok_off + t) * H * (two ? 2 : 1)] (BERTScore):
// fp16, or (two) the two-part image [hi | lo*64]
hipError_t launch_embed_out(const float* x32, const float2* stats, const float* g, const float* b,
                            SeqMeta sm, int s0, int s1, int row0, int H, f16* out, hipStream_t st,
                            const f16* himg = nullptr, bool two = false);
// max_len: longest sequence of the launch (0 = unknown): the 16x16x32 kernel serves chunks whose
// sequences all fit one 64-key block, the 32x32x16 kernel the others (fewer K/V reloads).
// dedup: qkv holds unique rows; sequence s, position t reads row (t == mask_pos ? urow_m : urow_h + t)
hipError_t launch_attention_full(const void* qkv, bool qkv32, SeqMeta sm, int s0, int s1, int row0,
                                 int H, int heads, f16* ctx, int kx, hipStream_t st, bool dedup = false,
                                 int max_len = 0);
// resq = LN(x32[query row]) (x32 pre-LN, with its row statistics and LN weight / bias)
hipError_t launch_attention_query(const void* qkv, bool qkv32, const float* x32, const float2* stats,
                                  const float* g, const float* b, SeqMeta sm, int s0, int s1,
                                  int row0, int H, int heads, f16* ctxq, float* resq, int kx,
                                  hipStream_t st, const void* qd = nullptr, const f16* himg = nullptr);
// dst[s - s0] = src[row of sequence s's query position], ld halfs per row
hipError_t launch_gather_query_rows(const f16* src, int ld, SeqMeta sm, int s0, int s1, int row0, f16* dst,
                                   hipStream_t st);
hipError_t launch_gather_labels(const int* tok, SeqMeta sm, int s0, int s1, int* lab,
                                hipStream_t st);
hipError_t launch_lse_finalize(const float2* part, int n_parts, const float* label_logit,
                               int rows, float* out, hipStream_t st);
hipError_t launch_cls_linear(const float* h, int rows, int H, const float* w, const float* b,
                             float* out, hipStream_t st);
hipError_t launch_segsum_f64(const float* row_lp, const int* hyp_seq_off, int n_hyp, double* out,
                             hipStream_t st);
