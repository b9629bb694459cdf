// Integer/fp64 kernels of the rerank stage (gfx950):
//
//  pairwise_edit  RMBR CER utility (RMBR/utility_functions.py:28-33 -> jiwer.cer per ordered
//                 pair, RMBR/mbr.py:8-16): Levenshtein matrix of every utterance's N-best,
//                 computed once per unordered pair (ed is symmetric) and reused for every
//                 top-k length of RMBR/main.py:15-35.
//  ref_edit       ed(reference, hypothesis) per hypothesis: the corpus-CER numerator table
//                 behind jiwer.cer(ref_list, pred_list) (rescore.py:40,118).
//  mbr_scores     RMBR/mbr.py:17-22 scores + argmax with torch-CPU float32 summation order.
//  fuse_rerank    rescore.py:47-58 over the whole weight grid at once (fp64, no contraction,
//                 same operation order), first-max argmax.
//  corpus_edits   per-weight sum of the argmax hypotheses' edits (exact integer CER numerator).
//
// Edit distance: Myers/Hyyro bit-parallel, one 64-bit word when the shorter string has <= 64
// symbols, else the blocked form (words of 64 pattern rows, up to RS_MAX_EDIT symbols).
#include "common.h"
#include "../../include/rescore.h"

namespace {

__device__ int myers64(const int* __restrict__ a, int m, const int* __restrict__ b, int n) {
    // a: pattern (m <= 64), b: text.  Global edit distance (first DP row = 0..n).
    if (m == 0) return n;
    if (n == 0) return m;
    int pa[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) pa[i] = i < m ? a[i] : 0;
    const unsigned long long full = m == 64 ? ~0ull : ((1ull << m) - 1ull);
    const unsigned long long top = 1ull << (m - 1);
    unsigned long long Pv = full, Mv = 0ull;
    int score = m;
    for (int k = 0; k < n; ++k) {
        const int c = b[k];
        unsigned long long Eq = 0ull;
#pragma unroll
        for (int blk = 0; blk < 4; ++blk) {
            if (blk * 16 < m) {
#pragma unroll
                for (int i = 0; i < 16; ++i) Eq |= (unsigned long long)(pa[blk * 16 + i] == c) << (blk * 16 + i);
            }
        }
        Eq &= full;
        const unsigned long long Xv = Eq | Mv;
        const unsigned long long Xh = (((Eq & Pv) + Pv) ^ Pv) | Eq;
        unsigned long long Ph = Mv | ~(Xh | Pv);
        unsigned long long Mh = Pv & Xh;
        if (Ph & top) ++score;
        else if (Mh & top) --score;
        Ph = (Ph << 1) | 1ull;
        Mh <<= 1;
        Pv = (Mh | ~(Xv | Ph)) & full;
        Mv = Ph & Xv;
    }
    return score;
}

// Blocked Myers / Hyyro (the pattern cut into 64-row words, horizontal deltas carried from
// word to word): exact global edit distance for patterns of up to RS_MAX_EDIT symbols.  The
// bit-vector recurrence is O(ceil(m / 64) * n) word operations, but the per-word Eq masks are
// formed on the fly by comparing every pattern symbol with each text symbol, so the total is
// O(m * n) scalar compares (no Peq table: the alphabet is open-ended code points), and Pv / Mv
// (2 x 2 KiB per thread, dynamically indexed) live in scratch.  Only strings longer than 64
// symbols come here; ASR hypotheses of the C5 workload never do (myers64 above).
constexpr int RS_MAX_EDIT = 16384;
constexpr int RS_MAX_WORDS = RS_MAX_EDIT / 64;

__device__ int myers_blocked(const int* __restrict__ a, int m, const int* __restrict__ b, int n) {
    unsigned long long Pv[RS_MAX_WORDS], Mv[RS_MAX_WORDS];
    const int nw = (m + 63) >> 6;
    for (int w = 0; w < nw; ++w) { Pv[w] = ~0ull; Mv[w] = 0ull; }
    const unsigned long long top = 1ull << ((m - 1) & 63);   // last pattern row, in the last word
    int score = m;
    for (int k = 0; k < n; ++k) {
        const int c = b[k];
        int hin = 1;                                          // first DP row 0..n: delta +1
        for (int w = 0; w < nw; ++w) {
            const int base = w << 6, rows = min(64, m - base);
            unsigned long long Eq = 0ull;
            for (int i = 0; i < rows; ++i) Eq |= (unsigned long long)(a[base + i] == c) << i;
            const unsigned long long pv = Pv[w], mv = Mv[w];
            const unsigned long long Xv = Eq | mv;
            if (hin < 0) Eq |= 1ull;
            const unsigned long long Xh = (((Eq & pv) + pv) ^ pv) | Eq;
            unsigned long long Ph = mv | ~(Xh | pv);
            unsigned long long Mh = pv & Xh;
            const unsigned long long hb = w == nw - 1 ? top : (1ull << 63);
            const int hout = (Ph & hb) ? 1 : (Mh & hb) ? -1 : 0;
            Ph <<= 1;
            Mh <<= 1;
            if (hin < 0) Mh |= 1ull;
            else if (hin > 0) Ph |= 1ull;
            Pv[w] = Mh | ~(Xv | Ph);
            Mv[w] = Ph & Xv;
            hin = hout;
        }
        score += hin;
    }
    return score;
}

// exact for strings of up to RS_MAX_EDIT symbols on the shorter side; -1 beyond (the host
// wrappers reject such inputs before launching)
__device__ int edit_distance(const int* a, int na, const int* b, int nb) {
    if (na > nb) {  // pattern = shorter string (ed is symmetric)
        const int* t = a; a = b; b = t;
        int tn = na; na = nb; nb = tn;
    }
    if (na <= 64) return myers64(a, na, b, nb);
    if (na <= RS_MAX_EDIT) return myers_blocked(a, na, b, nb);
    return -1;
}

__global__ void __launch_bounds__(256)
pairwise_edit_kernel(const int* __restrict__ chars, const int* __restrict__ str_off,
                     const int* __restrict__ utt_off, const long long* __restrict__ mat_off,
                     int* __restrict__ ed) {
    const int u = blockIdx.x;
    const int s0 = utt_off[u], n = utt_off[u + 1] - s0;
    const long long mo = mat_off[u];
    const int npairs = n * (n - 1) / 2;
    for (int t = threadIdx.x; t < n; t += blockDim.x) ed[mo + (long long)t * n + t] = 0;
    for (int p = threadIdx.x; p < npairs; p += blockDim.x) {
        // unrank p -> (i, j), i < j, row-major over the strict upper triangle
        int i = 0, rem = p;
        while (rem >= n - 1 - i) { rem -= n - 1 - i; ++i; }
        const int j = i + 1 + rem;
        const int ai = str_off[s0 + i], aj = str_off[s0 + j];
        const int d = edit_distance(chars + ai, str_off[s0 + i + 1] - ai, chars + aj, str_off[s0 + j + 1] - aj);
        ed[mo + (long long)i * n + j] = d;
        ed[mo + (long long)j * n + i] = d;
    }
}

__global__ void ref_edit_kernel(const int* __restrict__ chars, const int* __restrict__ str_off,
                                const int* __restrict__ utt_off, const int* __restrict__ ref_chars,
                                const int* __restrict__ ref_off, int n_utt, int* __restrict__ out) {
    const int u = blockIdx.y;
    if (u >= n_utt) return;
    const int r0 = ref_off[u];
    // any number of hypotheses per utterance: strided over the blocks of grid.x
    for (int s = utt_off[u] + blockIdx.x * blockDim.x + threadIdx.x; s < utt_off[u + 1]; s += gridDim.x * blockDim.x)
        out[s] = edit_distance(ref_chars + r0, ref_off[u + 1] - r0, chars + str_off[s], str_off[s + 1] - str_off[s]);
}

// torch-CPU float32 Tensor.sum(-1) order for a contiguous row of n values (n < 512):
// ATen cascade_sum -> n < 8: row_sum with 4 interleaved accumulators; n >= 8: 8-wide
// vectors summed by row_sum (4 vector accumulators), scalar tail, then the 8 lanes.
template <class Get>
__device__ float torch_sum_f32(int n, Get get) {
    if (n <= 0) return 0.f;
    if (n < 8) {
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        const int sz = n / 4;
        for (int t = 0; t < sz; ++t)
            for (int k = 0; k < 4; ++k) acc[k] = __fadd_rn(acc[k], get(t * 4 + k));
        for (int i = sz * 4; i < n; ++i) acc[0] = __fadd_rn(acc[0], get(i));
        for (int k = 1; k < 4; ++k) acc[0] = __fadd_rn(acc[0], acc[k]);
        return acc[0];
    }
    const int nv = n / 8;
    const int sz = nv / 4;
    float va[4][8];
    for (int k = 0; k < 4; ++k)
        for (int l = 0; l < 8; ++l) va[k][l] = 0.f;
    for (int t = 0; t < sz; ++t)
        for (int k = 0; k < 4; ++k)
            for (int l = 0; l < 8; ++l) va[k][l] = __fadd_rn(va[k][l], get((t * 4 + k) * 8 + l));
    for (int v = sz * 4; v < nv; ++v)
        for (int l = 0; l < 8; ++l) va[0][l] = __fadd_rn(va[0][l], get(v * 8 + l));
    for (int k = 1; k < 4; ++k)
        for (int l = 0; l < 8; ++l) va[0][l] = __fadd_rn(va[0][l], va[k][l]);
    float fin = 0.f;
    for (int i = nv * 8; i < n; ++i) fin = __fadd_rn(fin, get(i));
    for (int l = 0; l < 8; ++l) fin = __fadd_rn(fin, va[0][l]);
    return fin;
}

__global__ void mbr_scores_kernel(const int* __restrict__ ed, const long long* __restrict__ mat_off,
                                  const int* __restrict__ utt_off, const int* __restrict__ len,
                                  int n_utt, int k, float* __restrict__ scores, int* __restrict__ argmax) {
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= n_utt) return;
    const int s0 = utt_off[u], n = utt_off[u + 1] - s0;
    const long long mo = mat_off[u];
    float best = 0.f;
    int bi = 0;
    for (int i = 0; i < k; ++i) {
        // sims in RMBR/mbr.py:10-13 order: j = 0..i-1, i+1..k-1; ref = hyp_j, cand = hyp_i
        auto get = [&](int t) -> float {
            const int j = t < i ? t : t + 1;
            const double c = (double)ed[mo + (long long)j * n + i] / (double)len[s0 + j];
            return (float)(1.0 - c);
        };
        const float sc = torch_sum_f32(k - 1, get);
        scores[(long long)u * k + i] = sc;
        if (i == 0 || sc > best) { best = sc; bi = i; }
    }
    argmax[u] = bi;
}

// RMBR mbr_decode with the BERTScore utility: sim(i, j) = P/R/F of cand hyp_i against
// ref hyp_j from the recall matrix (P(i|j) = R(j|i)), summed like the CER utility.
#pragma clang fp contract(off)
__global__ void mbr_scores_bs_kernel(const float* __restrict__ rmat, const long long* __restrict__ mat_off,
                                     const int* __restrict__ utt_off, int n_utt, int k, int which,
                                     float* __restrict__ scores, int* __restrict__ argmax) {
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= n_utt) return;
    const int n = utt_off[u + 1] - utt_off[u];
    const long long mo = mat_off[u];
    float best = 0.f;
    int bi = 0;
    for (int i = 0; i < k; ++i) {
        auto get = [&](int t) -> float {
            const int j = t < i ? t : t + 1;
            const float r = rmat[mo + (long long)i * n + j], p = rmat[mo + (long long)j * n + i];
            if (which == RS_BS_R) return r;
            if (which == RS_BS_P) return p;
            const float f = __fdiv_rn(__fmul_rn(__fmul_rn(2.0f, p), r), __fadd_rn(p, r));
            return f != f ? 0.f : f;              // bert_score: F.masked_fill(isnan(F), 0)
        };
        const float sc = torch_sum_f32(k - 1, get);
        scores[(long long)u * k + i] = sc;
        if (i == 0 || sc > best) { best = sc; bi = i; }
    }
    argmax[u] = bi;
}

#pragma clang fp contract(off)
__global__ void fuse_rerank_kernel(const double* __restrict__ am, const double* __restrict__ lm,
                                   const int* __restrict__ len, const int* __restrict__ utt_off,
                                   int n_utt, int n_best, const double* __restrict__ wgrid, int n_w,
                                   int mode, int* __restrict__ out) {
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    const int w = blockIdx.y;
    if (u >= n_utt || w >= n_w) return;
    const double wt = wgrid[w];
    const double a1 = 1.0 - wt;
    const int s0 = utt_off[u];
    const int n = min(n_best, utt_off[u + 1] - s0);
    double best = 0.0;
    int bi = 0;
    for (int i = 0; i < n; ++i) {
        const double L = (double)len[s0 + i];
        double a = __dmul_rn(a1, am[s0 + i]);
        double b = __dmul_rn(wt, lm[s0 + i]);
        if (mode == RS_FUSE_NORM) {
            a = __ddiv_rn(a, L);
            b = __ddiv_rn(b, L);
        } else if (mode == RS_FUSE_AM_NORM) {
            a = __ddiv_rn(a, L);
        }
        const double sc = __dadd_rn(a, b);
        // np.argmax: first maximal element; a NaN wins (numpy propagates NaN as max)
        if (i == 0 || sc > best || (sc != sc && best == best)) { best = sc; bi = i; }
    }
    out[(long long)w * n_utt + u] = bi;
}

__global__ void __launch_bounds__(256)
corpus_edits_kernel(const int* __restrict__ ed_ref, const int* __restrict__ utt_off,
                    const int* __restrict__ argmax, int n_utt, long long* __restrict__ edits) {
    const int w = blockIdx.x;
    __shared__ long long part[256];
    long long s = 0;
    for (int u = threadIdx.x; u < n_utt; u += 256) s += ed_ref[utt_off[u] + argmax[(long long)w * n_utt + u]];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) edits[w] = part[0];
}

}  // namespace

extern "C" {

int rs_pairwise_edit(const int32_t* d_chars, const int32_t* d_str_off, const int32_t* d_utt_off,
                     const int64_t* d_mat_off, int32_t n_utt, int32_t max_n, int32_t* d_ed, void* stream) {
    if (n_utt < 0 || max_n < 0) return RS_EARG;
    if (n_utt == 0) return RS_OK;
    (void)max_n;
    hipLaunchKernelGGL(pairwise_edit_kernel, dim3(n_utt), dim3(256), 0, (hipStream_t)stream, d_chars,
                       d_str_off, d_utt_off, (const long long*)d_mat_off, d_ed);
    return hipGetLastError() == hipSuccess ? RS_OK : RS_EHIP;
}

int rs_ref_edit(const int32_t* d_chars, const int32_t* d_str_off, const int32_t* d_utt_off,
                const int32_t* d_ref_chars, const int32_t* d_ref_off, int32_t n_utt, int32_t* d_ed_ref,
                void* stream) {
    if (n_utt < 0) return RS_EARG;
    if (n_utt == 0) return RS_OK;
    // 16 x 64 threads per utterance, hypotheses strided over them (any count)
    hipLaunchKernelGGL(ref_edit_kernel, dim3(16, n_utt), dim3(64), 0, (hipStream_t)stream, d_chars, d_str_off,
                       d_utt_off, d_ref_chars, d_ref_off, n_utt, d_ed_ref);
    return hipGetLastError() == hipSuccess ? RS_OK : RS_EHIP;
}

int rs_mbr_scores(const int32_t* d_ed, const int64_t* d_mat_off, const int32_t* d_utt_off,
                  const int32_t* d_len, int32_t n_utt, int32_t k, float* d_scores, int32_t* d_argmax,
                  void* stream) {
    if (n_utt < 0 || k < 1 || k > 512) return RS_EARG;
    if (n_utt == 0) return RS_OK;
    hipLaunchKernelGGL(mbr_scores_kernel, dim3((n_utt + 63) / 64), dim3(64), 0, (hipStream_t)stream, d_ed,
                       (const long long*)d_mat_off, d_utt_off, d_len, n_utt, k, d_scores, d_argmax);
    return hipGetLastError() == hipSuccess ? RS_OK : RS_EHIP;
}

int rs_mbr_scores_bs(const float* d_rmat, const int64_t* d_mat_off, const int32_t* d_utt_off, int32_t n_utt,
                     int32_t k, int32_t which, float* d_scores, int32_t* d_argmax, void* stream) {
    if (n_utt < 0 || k < 1 || k > 512 || which < RS_BS_P || which > RS_BS_F) return RS_EARG;
    if (n_utt == 0) return RS_OK;
    hipLaunchKernelGGL(mbr_scores_bs_kernel, dim3((n_utt + 63) / 64), dim3(64), 0, (hipStream_t)stream, d_rmat,
                       (const long long*)d_mat_off, d_utt_off, n_utt, k, which, d_scores, d_argmax);
    return hipGetLastError() == hipSuccess ? RS_OK : RS_EHIP;
}

int rs_fuse_rerank(const double* d_am, const double* d_lm, const int32_t* d_len, const int32_t* d_utt_off,
                   int32_t n_utt, int32_t n_best, const double* d_w, int32_t n_w, int32_t mode,
                   int32_t* d_argmax, void* stream) {
    if (n_utt < 0 || n_w < 0 || n_best < 1 || mode < 0 || mode > 2) return RS_EARG;
    if (n_utt == 0 || n_w == 0) return RS_OK;
    hipLaunchKernelGGL(fuse_rerank_kernel, dim3((n_utt + 255) / 256, n_w), dim3(256), 0, (hipStream_t)stream,
                       d_am, d_lm, d_len, d_utt_off, n_utt, n_best, d_w, n_w, mode, d_argmax);
    return hipGetLastError() == hipSuccess ? RS_OK : RS_EHIP;
}

int rs_corpus_edits(const int32_t* d_ed_ref, const int32_t* d_utt_off, const int32_t* d_argmax, int32_t n_utt,
                    int32_t n_w, int64_t* d_edits, void* stream) {
    if (n_utt < 0 || n_w < 0) return RS_EARG;
    if (n_w == 0) return RS_OK;
    hipLaunchKernelGGL(corpus_edits_kernel, dim3(n_w), dim3(256), 0, (hipStream_t)stream, d_ed_ref, d_utt_off,
                       d_argmax, n_utt, (long long*)d_edits);
    return hipGetLastError() == hipSuccess ? RS_OK : RS_EHIP;
}

}  // extern "C"
