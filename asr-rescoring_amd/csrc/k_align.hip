// Levenshtein alignment with backtrace (espnet_data/preprocess/align.py:5-97,
// levenshtein_distance_alignment, used by Nbest_Align/preprocess.py:92-108 and
// CorrectBart/get_feature.py:111-127).
//
// Rules of the reference (restated from the review of that function; known answers in
// SURVEY §4 / align.py:12-18):
//   * both token lists get a start sentinel: cost matrix C[0..Lh][0..Lr], rows = hypothesis
//     tokens, columns = reference tokens; C[i][0] = i labelled D, C[0][j] = j labelled I;
//   * hyp[i-1] == ref[j-1]: C = C[i-1][j-1], labelled U (no min over the alternatives);
//   * else S = C[i-1][j-1] + 1 is the candidate, replaced only by a STRICTLY smaller
//     I = C[i][j-1] + 1, then by a strictly smaller D = C[i-1][j] + 1;
//   * traceback from (Lh, Lr): U / S consume both tokens, D emits ref "*" and the hyp token,
//     I emits the ref token and hyp "*"; the three lists are reversed at the end.
//
// gfx950 design: one wave per (ref, hyp) pair.  The DP runs as an anti-diagonal wavefront —
// lane l owns hypothesis row i = 64*strip + 1 + l and at step t computes column j = t - l, so
// a cell's up / diagonal neighbours are lane l-1's last two values (two __shfl_up) and its left
// neighbour is the lane's own last value; rows beyond 64 are strip-mined, the strip's last row
// handed down through LDS.  Labels (one byte per cell) go to a caller-sized global scratch;
// lane 0 walks the traceback, all lanes then reverse the pair's output in place.
#include <string>
#include "common.h"
#include "../../include/rescore.h"

namespace {

constexpr int RS_ALIGN_MAX = 4096;      // tokens per side (LDS hand-down rows: 2 x 16 KiB)

__global__ void __launch_bounds__(64)
align_kernel(const int* __restrict__ ref, const int* __restrict__ ref_off, const int* __restrict__ hyp,
             const int* __restrict__ hyp_off, const long long* __restrict__ lab_off, unsigned char* __restrict__ lab,
             const long long* __restrict__ out_off, signed char* __restrict__ ops, int* __restrict__ ref_idx,
             int* __restrict__ hyp_idx, int* __restrict__ n_out) {
    // C[row above the strip][0..Lr] (read) and the strip's last row (written): two buffers, so
    // the last row's writes never meet lane 0's reads of the row above
    __shared__ int rows[2][RS_ALIGN_MAX + 1];
    const int p = blockIdx.x, lane = threadIdx.x;
    const int r0 = ref_off[p], Lr = ref_off[p + 1] - r0;
    const int h0 = hyp_off[p], Lh = hyp_off[p + 1] - h0;
    unsigned char* L = lab + lab_off[p];    // L[i * (Lr + 1) + j], 1 <= i <= Lh, 1 <= j <= Lr
    const int W = Lr + 1;
    for (int j = lane; j <= Lr; j += 64) rows[0][j] = j;  // C[0][j] = j
    __syncthreads();
    for (int s0 = 0; s0 < Lh; s0 += 64) {
        const int* top = rows[(s0 >> 6) & 1];
        int* bot = rows[((s0 >> 6) & 1) ^ 1];
        const int i = s0 + 1 + lane;                      // this lane's row
        const bool row_ok = i <= Lh;
        const int hv = row_ok ? hyp[h0 + i - 1] : 0;
        const int last = min(63, Lh - 1 - s0);            // lane holding the strip's last row
        int cur = i, prv = i - 1;                         // C[i][j-1], C[i][j-2] (j = 1: C[i][0] = i)
        for (int t = 1; t <= Lr + 63; ++t) {
            const int j = t - lane;
            int up = __shfl_up(cur, 1), dg = __shfl_up(prv, 1);
            if (lane == 0 && j >= 1 && j <= Lr) {          // row above the strip from LDS
                up = top[j];
                dg = top[j - 1];
            }
            if (row_ok && j >= 1 && j <= Lr) {
                int v;
                unsigned char lb;
                if (hv == ref[r0 + j - 1]) {
                    v = dg;
                    lb = 0;                                // U
                } else {
                    v = dg + 1;
                    lb = 1;                                // S
                    if (cur + 1 < v) { v = cur + 1; lb = 2; }   // I (left)
                    if (up + 1 < v) { v = up + 1; lb = 3; }     // D (up)
                }
                L[(long long)i * W + j] = lb;
                prv = cur;
                cur = v;
                if (lane == last) bot[j] = v;              // hand the strip's last row down
            }
        }
        if (lane == 0) bot[0] = min(s0 + 64, Lh);          // C[last row][0]
        __syncthreads();
    }
    // traceback (lane 0), written back to front, then reversed by all lanes
    const long long o0 = out_off[p];
    __shared__ int cnt;
    // the labels other lanes stored are read by lane 0: one wave, so retiring its stores
    // (workgroup-scope fence: s_waitcnt vmcnt(0)) orders them before the loads
    __threadfence_block();
    __syncthreads();
    if (lane == 0) {
        int i = Lh, j = Lr, n = 0;
        while (i > 0 || j > 0) {
            const int lb = i == 0 ? 2 : j == 0 ? 3 : L[(long long)i * W + j];
            int ri = -1, hi = -1;
            if (lb <= 1) { ri = j - 1; hi = i - 1; --i; --j; }
            else if (lb == 2) { ri = j - 1; --j; }
            else { hi = i - 1; --i; }
            ops[o0 + n] = (signed char)lb;
            ref_idx[o0 + n] = ri;
            hyp_idx[o0 + n] = hi;
            ++n;
        }
        cnt = n;
        n_out[p] = n;
    }
    __threadfence_block();
    __syncthreads();
    const int n = cnt;
    for (int k = lane; k < n / 2; k += 64) {
        const long long a = o0 + k, b = o0 + n - 1 - k;
        const signed char oa = ops[a], ob = ops[b];
        const int ra = ref_idx[a], rb = ref_idx[b], ha = hyp_idx[a], hb = hyp_idx[b];
        ops[a] = ob; ops[b] = oa;
        ref_idx[a] = rb; ref_idx[b] = ra;
        hyp_idx[a] = hb; hyp_idx[b] = ha;
    }
}

}  // namespace

int rs_fail(int code, const std::string& msg);

extern "C" {

int rs_align(const int32_t* d_ref, const int32_t* d_ref_off, const int32_t* d_hyp, const int32_t* d_hyp_off,
             int32_t n_pairs, const int64_t* d_lab_off, uint8_t* d_lab, const int64_t* d_out_off, int8_t* d_ops,
             int32_t* d_ref_idx, int32_t* d_hyp_idx, int32_t* d_n, int32_t max_len, void* stream) {
    if (n_pairs < 0 || (n_pairs > 0 && (!d_ref_off || !d_hyp_off || !d_lab_off || !d_lab || !d_out_off || !d_ops ||
                                         !d_ref_idx || !d_hyp_idx || !d_n)))
        return rs_fail(RS_EARG, "rs_align: null argument");
    if (max_len > RS_ALIGN_MAX) return rs_fail(RS_EUNSUP, "rs_align: token lists are limited to 4096 tokens");
    if (n_pairs == 0) return RS_OK;
    hipLaunchKernelGGL(align_kernel, dim3(n_pairs), dim3(64), 0, (hipStream_t)stream, d_ref, d_ref_off, d_hyp,
                       d_hyp_off, (const long long*)d_lab_off, d_lab, (const long long*)d_out_off, (signed char*)d_ops,
                       d_ref_idx, d_hyp_idx, d_n);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? RS_OK : rs_fail(RS_EHIP, hipGetErrorString(e));
}

}  // extern "C"
