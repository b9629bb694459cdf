// BERTScore MBR utility (RMBR/utility_functions.py:9-22, which calls bert_score.score;
// bert_score is not installed here — its published algorithm, greedy_cos_idf with
// idf=False, is restated in oracle/bertscore_ref.py).
//
// For every utterance and every ordered pair (cand i, ref j) of its hypotheses:
//   R(i|j) = (1 / (T_j - 2)) * sum_{t in j, t != [CLS],[SEP]}  max_{s in i} cos(e_s, e_t)
// (the max runs over all of cand i's tokens, [CLS]/[SEP] included: bert_score's masks are the
// attention masks, only the idf weights drop the special tokens).  P(i|j) = R(j|i).
//
// bs_recall_kernel: one workgroup per work item = a run of whole ref hypotheses whose tokens
// fit one 64-column tile (32 in the split-operand form; a longer hypothesis is walked in
// sub-tiles).  The tile's
// ref embeddings sit in LDS; 8 waves stream the utterance's cand rows (packed, 32 rows per
// MFMA tile, v_mfma_f32_32x32x16_f16, fp32 accumulation) straight from global memory, fold
// each tile's 32x64 cosines into per-(cand hypothesis, column) maxima with LDS ordered-int
// atomic max (exact, order-independent), then reduce the maxima of each ref hypothesis'
// interior columns in column order.  A second matrix (rmat0, optional) takes each maximum as
// max(m, 0): bert_score multiplies the cosines by the pair batch's pad masks, so when the cand
// is shorter than the longest cand of its batch a padded position offers a cosine of 0 to the
// max (bertscore.py picks R or R0 per pair from the caller's batch layout).
#include "common.h"

namespace {

__device__ __forceinline__ unsigned f2key(float f) {
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(unsigned k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

template <int NV, bool TWO>
struct BsCfg {
    static constexpr int H = NV * 256;
    static constexpr int LDB = H + 8;          // +16 B per row: conflict-free ds_read_b128
    static constexpr int COLS = TWO ? 32 : 64; // ref columns per tile (TWO: hi and lo images in LDS)
    static constexpr int NG = NV <= 3 ? 128 : 64;
    static constexpr size_t smem = (size_t)COLS * LDB * 2 * (TWO ? 2 : 1) + (size_t)NG * COLS * 4;
};

// TWO (fp16x3 mode): emb rows are two-part images [hi | lo*64] (2H halves), and every cosine
// is the three significant products hi.hi + (hi/64).lo + lo.(hi/64) accumulated in fp32 on the
// fp16 MFMA (the power-of-two factors cancel exactly, as in gemm_x3s): fp32-class cosines
// (~2^-22 relative), like bert_score's fp32 embeddings and matmul.
template <int NV, bool TWO>
__global__ void __launch_bounds__(512)
bs_recall_kernel(const f16* __restrict__ emb, const int* __restrict__ hyp_off,
                 const int* __restrict__ utt_off, const long long* __restrict__ mat_off,
                 const int4* __restrict__ items, float* __restrict__ rmat, float* __restrict__ rmat0) {
    using C = BsCfg<NV, TWO>;
    constexpr int H = C::H, LDB = C::LDB, NG = C::NG, NKB = H / 64, COLS = C::COLS;
    constexpr int NPART = TWO ? 2 : 1, LDE = H * NPART;     // halves per embedding row
    extern __shared__ __attribute__((aligned(16))) char smem[];
    f16* sB = (f16*)smem;                          // [part][COLS][LDB]
    unsigned* cm = (unsigned*)(smem + (size_t)COLS * LDB * 2 * NPART);

    const int4 it = items[blockIdx.x];
    const int u = it.x, j0 = it.y, j1 = it.z;
    const int h0 = utt_off[u], n = utt_off[u + 1] - h0;
    const int* ho = hyp_off + h0;                 // ho[0..n]: token offsets of the utterance
    const long long mo = mat_off[u];
    const int cbeg = ho[j0], cend = ho[j1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hf = lane >> 5, l32 = lane & 31;
    const half8 down = (half8)(f16)X3_DOWN;

    for (int cs = cbeg; cs < cend; cs += COLS) {
        const int ncol = min(COLS, cend - cs);
        __syncthreads();                          // previous sub-tile's LDS readers are done
        for (int q = tid; q < NPART * COLS * (H / 8); q += 512) {
            const int pr = q / (COLS * (H / 8)), rq = q % (COLS * (H / 8));
            const int r = rq / (H / 8), c8 = rq % (H / 8);
            half8 v = {};
            if (r < ncol) v = *(const half8*)(emb + (size_t)(cs + r) * LDE + pr * H + c8 * 8);
            *(half8*)(sB + ((size_t)pr * COLS + r) * LDB + c8 * 8) = v;
        }
        for (int g0 = 0; g0 < n; g0 += NG) {
            const int g1 = min(n, g0 + NG);
            for (int q = tid; q < NG * COLS; q += 512) cm[q] = 0u;
            __syncthreads();
            const int r0 = ho[g0], r1 = ho[g1];
            int hc = g0;                          // this wave's hypothesis cursor (rows only grow)
            for (int rb = r0 + 32 * wave; rb < r1; rb += 32 * 8) {
                // K permutation shared by A and B: block kb, lane half hf, step s covers
                // k = 64 kb + 32 hf + 8 s + [0, 8), so each lane reads 64 contiguous bytes per block
                const int arow = rb + l32 < r1 ? rb + l32 : r0;   // rows past r1 are never folded
                const f16* ap = emb + (size_t)arow * LDE + 32 * hf;
                const f16* bp = sB + l32 * LDB + 32 * hf;
                f32x16 acc0 = {}, acc1 = {};
                half8 a[NPART][4], an[NPART][4];
#pragma unroll
                for (int pr = 0; pr < NPART; ++pr)
#pragma unroll
                    for (int s = 0; s < 4; ++s) a[pr][s] = *(const half8*)(ap + pr * H + 8 * s);
#pragma unroll
                for (int kb = 0; kb < NKB; ++kb) {
                    if (kb + 1 < NKB) {
#pragma unroll
                        for (int pr = 0; pr < NPART; ++pr)
#pragma unroll
                            for (int s = 0; s < 4; ++s) an[pr][s] = *(const half8*)(ap + pr * H + (kb + 1) * 64 + 8 * s);
                    }
#pragma unroll
                    for (int s = 0; s < 4; ++s) {
                        if constexpr (TWO) {
                            const half8 bh = *(const half8*)(bp + kb * 64 + 8 * s);
                            const half8 bl = *(const half8*)(bp + (size_t)COLS * LDB + kb * 64 + 8 * s);
                            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0][s], bh, acc0, 0, 0, 0);
                            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0][s] * down, bl, acc0, 0, 0, 0);
                            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[NPART - 1][s], bh * down, acc0, 0, 0, 0);
                        } else {
                            const half8 b0 = *(const half8*)(bp + kb * 64 + 8 * s);
                            const half8 b1 = *(const half8*)(bp + 32 * LDB + kb * 64 + 8 * s);
                            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0][s], b0, acc0, 0, 0, 0);
                            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0][s], b1, acc1, 0, 0, 0);
                        }
                    }
                    if (kb + 1 < NKB) {
#pragma unroll
                        for (int pr = 0; pr < NPART; ++pr)
#pragma unroll
                            for (int s = 0; s < 4; ++s) a[pr][s] = an[pr][s];
                    }
                }
                // lane holds column l32 (+32 in acc1), rows 8(v/4) + 4hf + v%4 of the tile
                while (ho[hc + 1] <= rb) ++hc;
                for (int h = hc; h < g1 && ho[h] < rb + 32; ++h) {
                    const int lo = ho[h] - rb, hi = ho[h + 1] - rb;
                    float m0 = -INFINITY, m1 = -INFINITY;
#pragma unroll
                    for (int v = 0; v < 16; ++v) {
                        const int row = 8 * (v >> 2) + 4 * hf + (v & 3);
                        const bool in = row >= lo && row < hi;
                        m0 = in ? fmaxf(m0, acc0[v]) : m0;
                        if constexpr (!TWO) m1 = in ? fmaxf(m1, acc1[v]) : m1;
                    }
                    m0 = fmaxf(m0, __shfl_xor(m0, 32));
                    if constexpr (!TWO) m1 = fmaxf(m1, __shfl_xor(m1, 32));
                    if (hf == 0) {
                        unsigned* row = cm + (h - g0) * COLS;
                        if (l32 < ncol) atomicMax(row + l32, f2key(m0));
                        if constexpr (!TWO) {
                            if (l32 + 32 < ncol) atomicMax(row + 32 + l32, f2key(m1));
                        }
                    }
                }
            }
            __syncthreads();
            // R(i|j) over this sub-tile's interior columns of j, summed in column order
            const int nj = j1 - j0;
            for (int q = tid; q < (g1 - g0) * nj; q += 512) {
                const int i = g0 + q / nj, j = j0 + q % nj;
                const int tb = ho[j], te = ho[j + 1];
                const int Tj = te - tb, Ti = ho[i + 1] - ho[i];
                float* dst = rmat + mo + (long long)i * n + j;
                float* dst0 = rmat0 ? rmat0 + mo + (long long)i * n + j : nullptr;
                float acc = cs == cbeg ? 0.f : *dst;
                float acc0 = cs == cbeg || !dst0 ? 0.f : *dst0;
                if (Tj > 2 && Ti > 2) {
                    const float w = 1.0f / (float)(Tj - 2);
                    const int lo = max(tb + 1, cs), hi = min(te - 1, cs + COLS);
                    for (int t = lo; t < hi; ++t) {
                        const float v = key2f(cm[(i - g0) * COLS + (t - cs)]);
                        acc += v * w;
                        acc0 += fmaxf(v, 0.f) * w;
                    }
                } else {
                    acc = acc0 = 0.f;             // bert_score: empty cand or ref -> P = R = 0
                }
                *dst = acc;
                if (dst0) *dst0 = acc0;
            }
            __syncthreads();                      // cm is cleared by the next group
        }
    }
}

template <int NV, bool TWO>
hipError_t launch_bs(const f16* emb, const int* hyp_off, const int* utt_off, const long long* mat_off,
                     const int4* items, int n_items, float* rmat, float* rmat0, hipStream_t st) {
    // set every launch (cheap; a process-wide "done" flag would miss a second device)
    hipError_t e = hipFuncSetAttribute((const void*)bs_recall_kernel<NV, TWO>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)(BsCfg<NV, TWO>::smem));
    if (e != hipSuccess) return e;
    constexpr size_t smem = BsCfg<NV, TWO>::smem;
    hipLaunchKernelGGL((bs_recall_kernel<NV, TWO>), dim3(n_items), dim3(512), smem, st, emb, hyp_off, utt_off, mat_off,
                       items, rmat, rmat0);
    return hipGetLastError();
}

}  // namespace

int bertscore_cols(bool two) { return two ? BsCfg<1, true>::COLS : BsCfg<1, false>::COLS; }

hipError_t launch_bertscore_recall(const f16* emb, int H, const int* hyp_off, const int* utt_off,
                                   const long long* mat_off, const int4* items, int n_items, float* rmat,
                                   float* rmat0, hipStream_t st, bool two) {
    if (n_items <= 0) return hipSuccess;
#define RS_BS(NV)                                                                                          \
    return two ? launch_bs<NV, true>(emb, hyp_off, utt_off, mat_off, items, n_items, rmat, rmat0, st)       \
               : launch_bs<NV, false>(emb, hyp_off, utt_off, mat_off, items, n_items, rmat, rmat0, st)
    switch (H) {
        case 256: RS_BS(1);
        case 512: RS_BS(2);
        case 768: RS_BS(3);
        case 1024: RS_BS(4);
        default: return hipErrorInvalidValue;
    }
#undef RS_BS
}
