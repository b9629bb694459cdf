// fp16 MFMA GEMM for the BERT projections: C[M,N] = A[M,K] . W[N,K]^T (+ fused epilogue).
//
// Replaces the nn.Linear calls of transformers modeling_bert.py (Q/K/V :154-156 fused into
// one [3H,H] GEMM, BertSelfOutput :282-293, BertIntermediate :325-337, BertOutput :340-351,
// BertPredictionHeadTransform :466-480, tied decoder :483-496 with the log-softmax of
// MLM_PLL/main.py:101-105 fused as an online logsumexp epilogue).
//
// gfx950 design:
//  * v_mfma_f32_32x32x16_f16, fp32 accumulators; A and W both K-contiguous, so A and B
//    fragments are the same 16-byte ds_read_b128 pattern (lane l: row l&31, k-chunk l>>5).
//  * BK = 64 (128-byte tile rows), two LDS stages filled by global_load_lds_dwordx4
//    (1 KiB = 8 rows per wave-instruction).  The LDS image is written lane-linear, so the
//    XOR swizzle (chunk ^= (row>>1)&7) is applied to the per-lane global SOURCE address and
//    to the ds_read address (the same involution): conflict-free ds_read_b128 for the
//    16-lane groups of a 32-row fragment read.
//  * XCD-aware bijective block remap: consecutive tiles (same A row panel) share an XCD L2.
#include "common.h"

namespace {

constexpr int BK = 64;

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

template <int BM, int BN, int WM, int WN, int EPI>
__global__ void __launch_bounds__(WM * WN * 64)
gemm_f16_kernel(const f16* __restrict__ A, const f16* __restrict__ W, int K, int n_tiles_n,
                EpiArgs ep) {
    constexpr int NW = WM * WN;
    constexpr int A_BYTES = BM * BK * 2;
    constexpr int STAGE = (BM + BN) * BK * 2;
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int TM = WTM / 32, TN = WTN / 32;
    constexpr int A_PIECES = BM / 8, PIECES = (BM + BN) / 8;
    static_assert(PIECES % NW == 0, "pieces per wave");
    constexpr int PPW = PIECES / NW;

    extern __shared__ __attribute__((aligned(16))) char smem[];

    // bijective XCD remap (blocks b and b+8 share an XCD on the observed dispatch)
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, pos = bid >> 3, q = nwg >> 3, r = nwg & 7;
    const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
    const int tm = wgid / n_tiles_n, tn = wgid - tm * n_tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;

    // per-lane global source pointers of the pieces this wave stages (k0 = 0)
    const f16* src[PPW];
    int ldsoff[PPW];
#pragma unroll
    for (int p = 0; p < PPW; ++p) {
        const int piece = p * NW + wave;
        const int lrow = lane >> 3, pc = lane & 7;
        if (piece < A_PIECES) {
            const int row = piece * 8 + lrow;
            src[p] = A + (size_t)(m0 + row) * K + swz(row, pc) * 8;
        } else {
            const int row = (piece - A_PIECES) * 8 + lrow;
            src[p] = W + (size_t)(n0 + row) * K + swz(row, pc) * 8;
        }
        ldsoff[p] = piece * 1024;
    }

    auto stage = [&](int buf, int k0) {
#pragma unroll
        for (int p = 0; p < PPW; ++p) {
            __builtin_amdgcn_global_load_lds(
                (const void*)(src[p] + k0),
                (__attribute__((address_space(3))) void*)(smem + buf * STAGE + ldsoff[p]), 16, 0, 0);
        }
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x16){};

    const int nk = K / BK;
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    const int frow = lane & 31, fh = lane >> 5;
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) stage(cur ^ 1, (kt + 1) * BK);
        const char* sA = smem + cur * STAGE;
        const char* sB = sA + A_BYTES;
#pragma unroll
        for (int s = 0; s < BK / 16; ++s) {
            half8 af[TM], bf[TN];
            const int lc = 2 * s + fh;
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int row = wm * WTM + i * 32 + frow;
                af[i] = *(const half8*)(sA + row * 128 + (swz(row, lc) << 4));
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int row = wn * WTN + j * 32 + frow;
                bf[j] = *(const half8*)(sB + row * 128 + (swz(row, lc) << 4));
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    // ---------------- epilogue (C/D layout: col = lane&31, row = (r&3)+8(r>>2)+4(lane>>5))
    const int rbase = m0 + wm * WTM + 4 * fh;
    const int cbase = n0 + wn * WTN + frow;
    if constexpr (EPI == EPI_LSE) {
        const int slab = (n0 + wn * WTN) / WTN;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = rbase + i * 32 + (r & 3) + 8 * (r >> 2);
                float v[TN];
                float mx = -INFINITY;
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int col = cbase + j * 32;
                    v[j] = col < ep.n_valid ? acc[i][j][r] + ep.bias[col] : -INFINITY;
                    mx = fmaxf(mx, v[j]);
                }
#pragma unroll
                for (int o = 16; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
                float sm = 0.f;
#pragma unroll
                for (int j = 0; j < TN; ++j) sm += (v[j] == -INFINITY) ? 0.f : __expf(v[j] - mx);
#pragma unroll
                for (int o = 16; o > 0; o >>= 1) sm += __shfl_xor(sm, o);
                if (row < ep.m_valid) {
                    if (frow == 0) ep.lse_part[(size_t)row * ep.n_parts + slab] = make_float2(mx, sm);
                    const int lab = ep.label[row];
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        if (cbase + j * 32 == lab) ep.label_logit[row] = v[j];
                }
            }
        }
    } else {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int col = cbase + j * 32;
                const float bias = ep.bias[col];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = rbase + i * 32 + (r & 3) + 8 * (r >> 2);
                    if (row >= ep.m_valid) continue;
                    float x = acc[i][j][r] + bias;
                    const size_t o = (size_t)row * ep.ldc + col;
                    if constexpr (EPI == EPI_BIAS_F16) {
                        ((f16*)ep.out)[o] = (f16)x;
                    } else if constexpr (EPI == EPI_BIAS_F32) {
                        ((float*)ep.out)[o] = x;
                    } else if constexpr (EPI == EPI_GELU_F16) {
                        put_split((f16*)ep.out + (size_t)row * ep.ldc, col, ep.nlog, ep.kx, gelu_erf(x));
                    } else if constexpr (EPI == EPI_GELU_F32) {
                        ((float*)ep.out)[o] = gelu_erf(x);
                    } else {  // EPI_RES_F32
                        ((float*)ep.out)[o] = x + ep.res[o];
                    }
                }
            }
        }
    }
}

template <int BM, int BN, int WM, int WN, int EPI>
hipError_t launch_t(const f16* A, const f16* W, int M_pad, int N_pad, int K, const EpiArgs& ep,
                    hipStream_t st) {
    constexpr int smem = 2 * (BM + BN) * BK * 2;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)gemm_f16_kernel<BM, BN, WM, WN, EPI>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, smem);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    const int ntn = N_pad / BN;
    const int grid = (M_pad / BM) * ntn;
    hipLaunchKernelGGL((gemm_f16_kernel<BM, BN, WM, WN, EPI>), dim3(grid), dim3(WM * WN * 64),
                       smem, st, A, W, K, ntn, ep);
    return hipGetLastError();
}

}  // namespace

int gemm_row_align() { return 128; }

hipError_t launch_gemm(int epi, const f16* A, const f16* W, int M_pad, int N_pad, int K,
                       const EpiArgs& ep, hipStream_t st) {
    if (M_pad % 128 || N_pad % 128 || K % BK || M_pad <= 0) return hipErrorInvalidValue;
    switch (epi) {
        case EPI_BIAS_F16: return launch_t<128, 128, 2, 2, EPI_BIAS_F16>(A, W, M_pad, N_pad, K, ep, st);
        case EPI_GELU_F16: return launch_t<128, 128, 2, 2, EPI_GELU_F16>(A, W, M_pad, N_pad, K, ep, st);
        case EPI_GELU_F32: return launch_t<128, 128, 2, 2, EPI_GELU_F32>(A, W, M_pad, N_pad, K, ep, st);
        case EPI_RES_F32: return launch_t<128, 128, 2, 2, EPI_RES_F32>(A, W, M_pad, N_pad, K, ep, st);
        case EPI_LSE: return launch_t<128, 128, 2, 2, EPI_LSE>(A, W, M_pad, N_pad, K, ep, st);
        case EPI_BIAS_F32: return launch_t<128, 128, 2, 2, EPI_BIAS_F32>(A, W, M_pad, N_pad, K, ep, st);
    }
    return hipErrorInvalidValue;
}
