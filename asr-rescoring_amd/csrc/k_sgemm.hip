// fp32 GEMMs of the trainer: the forward projections, the input
// gradients and the weight gradients of every nn.Linear the reference trains
// (RescoreBert/main.py:104-150, MLM_PLL/main.py:89-97 through transformers' BertModel).
//
// The reference trains in fp32, so these run on the f32-input MFMA (v_mfma_f32_32x32x2_f32:
// exact f32, every result a k-ordered fmaf chain) rather than on the fp16 split-operand
// kernels of the scoring path.  One kernel serves the three operand forms a Linear's
// forward / backward needs, chosen by where k is contiguous in each operand:
//   forward  Y  = X  · Wᵀ   A = X  [M][K] (k contiguous)   B = W [N][K] (k contiguous)
//   dgrad    dX = dY · W    A = dY [M][N] (k contiguous)   B = W [N][K] (n contiguous)
//   wgrad    dW = dYᵀ· X    A = dY [M][N] (m contiguous)   B = X [M][K] (n contiguous)
// Tiles: 128×128 outputs per workgroup (4 waves, 64×64 each = 2×2 MFMA tiles of 32×32),
// BK = 32.  Both operands are staged as [k][row] LDS images (row stride 132 floats), so every
// fragment read is one ds_read_b32 over consecutive rows; k-contiguous sources are loaded as
// float4 along k and transposed by the LDS writes, row-contiguous ones go in as float4.  The
// next K-step's tiles are loaded into registers while this step's MFMAs run, and each MFMA
// step's fragments are read one step ahead.  (Measured on MI355X with tools/sgemm_bench.py
// over the training shapes — DESIGN §8 "Training": two LDS stages with source-oriented images
// and ds_read_b128 fragments, the same with a bank-split [k][row] stride, loads two K-steps
// ahead (RS_SGEMM_MODE=2), two stages with the next step's pieces interleaved into the MFMAs
// (RS_SGEMM_MODE=3) and launch-bounds occupancy 3–4 were all equal or slower.)
// Few output tiles (the weight gradients of a ~1k-token batch, the projections of a small
// batch) are split over K: each split writes its partial tile to a workspace and an ordered
// sum over the splits closes it — no float atomics, so a training step stays bitwise
// reproducible.
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "train.h"

namespace {

constexpr int SG_BM = 128, SG_BN = 128, SG_BK = 32, SG_LD = SG_BM + 4;
// row stride of an operand's [k][row] image: 130 (≡ 2 mod 64 banks) for k-contiguous sources,
// whose transposed scalar writes then hit 64 distinct banks per wave (132: two-way
// conflicts); 132 for row-contiguous ones (16-B aligned rows for the float4 writes)
template <bool KC>
constexpr int sg_ld() { return KC ? SG_BM + 2 : SG_BM + 4; }
typedef float f32x16 __attribute__((ext_vector_type(16)));

// Loads one operand's [rows 128] × [k 32] tile into registers (4 float4 per thread).
// KC: the source is [row][ld] with k contiguous; otherwise [k][ld] with rows contiguous.
template <bool KC>
__device__ __forceinline__ void sg_load(const float* __restrict__ src, int ld, int row0, int rows, int k0, int kend,
                                        float4 (&r)[4]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int idx = t + 256 * i;
        int row, k;
        if (KC) {
            row = idx >> 3;
            k = (idx & 7) * 4;
        } else {
            k = idx >> 5;
            row = (idx & 31) * 4;
        }
        const int gr = row0 + row, gk = k0 + k;
        // extents along the contiguous dimension are multiples of 4 (host-checked): a float4
        // is either wholly inside or wholly outside
        const bool ok = gr < rows && gk < kend;
        r[i] = ok ? (KC ? *(const float4*)(src + (size_t)gr * ld + gk) : *(const float4*)(src + (size_t)gk * ld + gr))
                  : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

// [k][row] LDS image: k-contiguous sources are transposed by the writes (4 ds_write_b32 per
// float4), row-contiguous ones go in as one ds_write_b128.  Piece i (0..3) of this thread.
template <bool KC>
__device__ __forceinline__ void sg_store_one(float* __restrict__ s, int i, const float4 v) {
    const int idx = threadIdx.x + 256 * i;
    if (KC) {
        const int row = idx >> 3, k = (idx & 7) * 4;
        constexpr int L = sg_ld<true>();
        s[(k + 0) * L + row] = v.x;
        s[(k + 1) * L + row] = v.y;
        s[(k + 2) * L + row] = v.z;
        s[(k + 3) * L + row] = v.w;
    } else {
        const int k = idx >> 5, row = (idx & 31) * 4;
        *(float4*)(s + k * sg_ld<false>() + row) = v;
    }
}

template <bool KC>
__device__ __forceinline__ void sg_store_lds(float* __restrict__ s, const float4 (&r)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) sg_store_one<KC>(s, i, r[i]);
}

// C[M][N] (+)= A·B over k in [z·kc, min(K, (z+1)·kc)) for split z = blockIdx.z.
// ws == nullptr: C = acc (+ C when accum).  Otherwise the partial goes to ws[z][M][N].
// MODE 1 (default): one LDS stage — store, barrier, MFMAs, barrier per K-step, the next
// step's global loads in flight under the MFMAs.  MODE 2: the same with loads two K-steps
// ahead (a second register set).  MODE 3: two LDS stages — the next step's tiles are
// written to the other stage between the second half of this step's MFMAs (one float4 piece
// after each group of four), one barrier per K-step.
template <bool AKC, bool BKC, int MODE>
__global__ void __launch_bounds__(256)
sgemm_f32_kernel(const float* __restrict__ A, int lda, const float* __restrict__ B, int ldb, float* __restrict__ C,
                 int ldc, int M, int N, int K, int kc, int accum, float* __restrict__ ws) {
    extern __shared__ __attribute__((aligned(16))) float sg_smem[];   // stages x (A image | B image)
    constexpr int SIMG = SG_BK * SG_LD, PF = MODE == 2 ? 2 : 1;
    float* As = sg_smem;
    float* Bs = sg_smem + SIMG;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int m0 = blockIdx.y * SG_BM, n0 = blockIdx.x * SG_BN;
    const int kb = blockIdx.z * kc, ke = min(K, kb + kc);
    const int wm = (w & 1) * 64, wn = (w >> 1) * 64;
    const int h = lane >> 5, c = lane & 31;

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // one K-step: stage the registers' tiles, refill them PF steps ahead, multiply
    auto kstep = [&](int k0, float4 (&ra)[4], float4 (&rb)[4]) {
        sg_store_lds<AKC>(As, ra);
        sg_store_lds<BKC>(Bs, rb);
        __syncthreads();
        const int kn = k0 + PF * SG_BK;
        if (kn < ke) {                         // tiles PF steps ahead in flight under the MFMAs
            sg_load<AKC>(A, lda, m0, M, kn, ke, ra);
            sg_load<BKC>(B, ldb, n0, N, kn, ke, rb);
        }
        // MFMA step kk, lane half h: k = 2 kk + h (the instruction's A[i][k = lane >> 5] map).
        // Fragments of step kk + 1 are read before step kk's MFMAs issue, so the LDS latency
        // runs under the MFMA pipe (hipcc otherwise waits lgkmcnt(0) before every step).
        constexpr int LA = sg_ld<AKC>(), LB = sg_ld<BKC>();
        const float* ap = As + h * LA + wm + c;
        const float* bp = Bs + h * LB + wn + c;
        float a0 = ap[0], a1 = ap[32], b0 = bp[0], b1 = bp[32];
#pragma unroll
        for (int kk = 0; kk < SG_BK / 2; ++kk) {
            float na0 = 0.f, na1 = 0.f, nb0 = 0.f, nb1 = 0.f;
            if (kk + 1 < SG_BK / 2) {
                const int oa = 2 * (kk + 1) * LA, ob = 2 * (kk + 1) * LB;
                na0 = ap[oa]; na1 = ap[oa + 32]; nb0 = bp[ob]; nb1 = bp[ob + 32];
            }
            __builtin_amdgcn_sched_barrier(0);   // keep the reads ahead of this step's MFMAs
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            a0 = na0; a1 = na1; b0 = nb0; b1 = nb1;
        }
        __syncthreads();
    };

    float4 ra[4], rb[4];
    sg_load<AKC>(A, lda, m0, M, kb, ke, ra);
    sg_load<BKC>(B, ldb, n0, N, kb, ke, rb);
    if constexpr (MODE == 3) {
        sg_store_lds<AKC>(sg_smem, ra);
        sg_store_lds<BKC>(sg_smem + SIMG, rb);
        __syncthreads();
        int cur = 0;
        for (int k0 = kb; k0 < ke; k0 += SG_BK) {
            const bool more = k0 + SG_BK < ke;
            if (more) {
                sg_load<AKC>(A, lda, m0, M, k0 + SG_BK, ke, ra);
                sg_load<BKC>(B, ldb, n0, N, k0 + SG_BK, ke, rb);
            }
            constexpr int LA = sg_ld<AKC>(), LB = sg_ld<BKC>();
            const float* ap = sg_smem + cur * 2 * SIMG + h * LA + wm + c;
            const float* bp = sg_smem + cur * 2 * SIMG + SIMG + h * LB + wn + c;
            float* nx = sg_smem + (cur ^ 1) * 2 * SIMG;
            float a0 = ap[0], a1 = ap[32], b0 = bp[0], b1 = bp[32];
#pragma unroll
            for (int kk = 0; kk < SG_BK / 2; ++kk) {
                float na0 = 0.f, na1 = 0.f, nb0 = 0.f, nb1 = 0.f;
                if (kk + 1 < SG_BK / 2) {
                    const int oa = 2 * (kk + 1) * LA, ob = 2 * (kk + 1) * LB;
                    na0 = ap[oa]; na1 = ap[oa + 32]; nb0 = bp[ob]; nb1 = bp[ob + 32];
                }
                __builtin_amdgcn_sched_barrier(0);
                acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
                acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
                acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
                acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
                if (kk >= 8 && more) {         // pieces 0-3 of A, then of B, half a step after their loads
                    const int i = kk - 8;
                    if (i < 4) sg_store_one<AKC>(nx, i, ra[i]);
                    else sg_store_one<BKC>(nx + SIMG, i - 4, rb[i - 4]);
                }
                __builtin_amdgcn_sched_barrier(0);
                a0 = na0; a1 = na1; b0 = nb0; b1 = nb1;
            }
            __syncthreads();
            cur ^= 1;
        }
    } else if constexpr (PF == 1) {
        for (int k0 = kb; k0 < ke; k0 += SG_BK) kstep(k0, ra, rb);
    } else {
        float4 ra2[4], rb2[4];
        if (kb + SG_BK < ke) {
            sg_load<AKC>(A, lda, m0, M, kb + SG_BK, ke, ra2);
            sg_load<BKC>(B, ldb, n0, N, kb + SG_BK, ke, rb2);
        }
        for (int k0 = kb; k0 < ke; k0 += SG_BK) {
            kstep(k0, ra, rb);                 // refills ra / rb with step k0 + 2 BK
#pragma unroll
            for (int i = 0; i < 4; ++i) {      // the next step's tiles are in the second set
                const float4 ta = ra[i], tb = rb[i];
                ra[i] = ra2[i]; rb[i] = rb2[i];
                ra2[i] = ta; rb2[i] = tb;
            }
        }
    }

    // D map of the 32x32 forms: column = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    float* P = ws ? ws + (size_t)blockIdx.z * M * N : nullptr;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int col = n0 + wn + 32 * j + c;
            if (col >= N) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (row >= M) continue;
                if (P) {
                    P[(size_t)row * N + col] = acc[i][j][r];
                } else {
                    float* o = C + (size_t)row * ldc + col;
                    *o = accum ? acc[i][j][r] + *o : acc[i][j][r];
                }
            }
        }
}

// C = sum over splits z = 0, 1, ... of ws[z] (+ C), in split order
__global__ void __launch_bounds__(256)
sgemm_splitk_sum_kernel(const float* __restrict__ ws, int splits, int M, int N, float* __restrict__ C, int ldc,
                        int accum) {
    const size_t MN = (size_t)M * N;
    const size_t i4 = ((size_t)blockIdx.x * 256 + threadIdx.x) * 4;   // N % 4 == 0: whole float4 rows
    if (i4 >= MN) return;
    float4 s = *(const float4*)(ws + i4);
    for (int z = 1; z < splits; ++z) {
        const float4 p = *(const float4*)(ws + (size_t)z * MN + i4);
        s.x += p.x; s.y += p.y; s.z += p.z; s.w += p.w;
    }
    const size_t row = i4 / N, col = i4 % N;
    float4* o = (float4*)(C + row * ldc + col);
    if (accum) {
        const float4 q = *o;
        s.x += q.x; s.y += q.y; s.z += q.z; s.w += q.w;
    }
    *o = s;
}

int sg_splits(int M, int N, int K, int* kc) {
    const int tiles = ((M + SG_BM - 1) / SG_BM) * ((N + SG_BN - 1) / SG_BN);
    const int steps = (K + SG_BK - 1) / SG_BK;
    int splits = 1;
    // up to ~512 workgroups (two per CU); each split costs a write + read of M·N partials.
    // RS_SGEMM_SPLIT_WG overrides the workgroup target (A/B knob).
    static const int target = [] {
        const char* v = getenv("RS_SGEMM_SPLIT_WG");
        return v ? std::max(1, atoi(v)) : 512;
    }();
    if (tiles < target) splits = std::max(1, std::min(std::min((target + tiles - 1) / tiles, steps / 4), 16));
    const int per = (steps + splits - 1) / splits;
    *kc = per * SG_BK;
    return (steps + per - 1) / per;
}

}  // namespace

size_t tr_sgemm_ws_floats(int M, int N, int K) {
    int kc = 0;
    const int s = sg_splits(M, N, K, &kc);
    return s > 1 ? (size_t)s * M * N : 0;
}

hipError_t tr_sgemm(int M, int N, int K, const float* A, int lda, bool a_kc, const float* B, int ldb, bool b_kc,
                    float* C, int ldc, int accum, float* ws, size_t ws_floats, hipStream_t s) {
    if (M <= 0 || N <= 0) return hipSuccess;
    // float4 loads along each operand's contiguous dimension and along C's rows (split-K sum)
    if (N % 4 || lda % 4 || ldb % 4 || ldc % 4 || (a_kc ? K % 4 : M % 4) || (b_kc && K % 4) ||
        ((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) % 16)
        return hipErrorInvalidValue;
    if (K <= 0) {   // empty reduction: C = 0 (+ C)
        if (accum) return hipSuccess;
        for (int r = 0; r < M; ++r) {
            hipError_t e = hipMemsetAsync(C + (size_t)r * ldc, 0, (size_t)N * 4, s);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    int kc = 0;
    const int splits = sg_splits(M, N, K, &kc);
    float* P = nullptr;
    if (splits > 1) {
        if (!ws || ws_floats < (size_t)splits * M * N) return hipErrorInvalidValue;
        P = ws;
    }
    const dim3 grid((N + SG_BN - 1) / SG_BN, (M + SG_BM - 1) / SG_BM, splits);
#define SG_LAUNCH(AK, BK_, MD)                                                                              \
    do {                                                                                                    \
        constexpr int smem = (MD == 3 ? 4 : 2) * SG_BK * SG_LD * 4;                                          \
        if (smem > 65536) {                                                                                 \
            static bool attr = false;                                                                       \
            if (!attr) {                                                                                    \
                hipError_t ea = hipFuncSetAttribute((const void*)sgemm_f32_kernel<AK, BK_, MD>,             \
                                                    hipFuncAttributeMaxDynamicSharedMemorySize, smem);      \
                if (ea != hipSuccess) return ea;                                                            \
                attr = true;                                                                                \
            }                                                                                               \
        }                                                                                                   \
        hipLaunchKernelGGL((sgemm_f32_kernel<AK, BK_, MD>), grid, dim3(256), smem, s, A, lda, B, ldb, C, ldc, \
                           M, N, K, kc, accum, P);                                                          \
    } while (0)
#define SG_FORMS(MD)                                  \
    if (a_kc && b_kc) SG_LAUNCH(true, true, MD);      \
    else if (a_kc) SG_LAUNCH(true, false, MD);        \
    else if (b_kc) SG_LAUNCH(false, true, MD);        \
    else SG_LAUNCH(false, false, MD);
    static const int mode = [] {                       // RS_SGEMM_MODE=2/3: A/B knob
        const char* v = getenv("RS_SGEMM_MODE");
        const int m = v ? atoi(v) : 1;
        return m == 2 || m == 3 ? m : 1;
    }();
    if (mode == 3) {
        SG_FORMS(3)
    } else if (mode == 2) {
        SG_FORMS(2)
    } else {
        SG_FORMS(1)
    }
#undef SG_FORMS
#undef SG_LAUNCH
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || splits == 1) return e;
    const size_t n4 = (size_t)M * N / 4;
    hipLaunchKernelGGL(sgemm_splitk_sum_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, P, splits, M, N, C,
                       ldc, accum);
    return hipGetLastError();
}

// Test / timing entry (not part of the scoring path): one trainer GEMM in the given operand
// form; the split-K workspace is a grow-only buffer kept across calls (single-threaded use).
// Returns 0 on success.
extern "C" int rs_debug_sgemm(int M, int N, int K, const float* A, int lda, int a_kc, const float* B, int ldb, int b_kc,
                              float* C, int ldc, int accum, void* stream) {
    static float* ws = nullptr;
    static size_t ws_cap = 0;
    const size_t wsf = tr_sgemm_ws_floats(M, N, K);
    if (wsf > ws_cap) {
        if (ws) {
            (void)hipDeviceSynchronize();
            (void)hipFree(ws);
        }
        ws = nullptr;
        ws_cap = 0;
        if (hipMalloc(&ws, wsf * 4) != hipSuccess) return -3;
        ws_cap = wsf;
    }
    hipError_t e = tr_sgemm(M, N, K, A, lda, a_kc != 0, B, ldb, b_kc != 0, C, ldc, accum, ws, ws_cap,
                            (hipStream_t)stream);
    return e == hipSuccess ? 0 : -2;
}
