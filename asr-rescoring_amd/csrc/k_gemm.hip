#include <atomic>
// fp16 MFMA GEMM for the BERT projections: C[M,N] = A[M,K] . W[N,K]^T (+ fused epilogue).
//
// Replaces the nn.Linear calls of transformers modeling_bert.py (Q/K/V :154-156 fused into
// one [3H,H] GEMM, BertSelfOutput :282-293, BertIntermediate :325-337, BertOutput :340-351,
// BertPredictionHeadTransform :466-480, tied decoder :483-496 with the log-softmax of
// MLM_PLL/main.py:101-105 fused as an online logsumexp epilogue).
//
// gfx950 design:
//  * v_mfma_f32_32x32x16_f16, fp32 accumulators, operands SWAPPED (D = W_tile . A_tile^T):
//    the accumulator's lane index is the output ROW and its registers run along the output
//    COLUMNS, so every lane owns 4 consecutive columns of a row -> 16-byte epilogue stores,
//    16-byte bias/residual loads, and row reductions (decoder logsumexp) mostly in-register.
//  * A and W are both K-contiguous: both fragments are one ds_read_b128 (lane l: row l&31,
//    k-chunk l>>5).  BK = 64 (128-byte LDS tile rows).
//  * LDS ring of NSTAGE stages filled by global_load_lds_dwordx4 (1 KiB = 8 rows per
//    wave-instruction); counted `s_waitcnt vmcnt` + raw s_barrier (one per K-step) keep the
//    next stage's DMA in flight across the barrier (a __syncthreads() would drain it).
//    The LDS image is lane-linear, so the XOR swizzle (chunk ^= (row>>1)&7) goes on the
//    per-lane global SOURCE address and on the ds_read address: conflict-free b128 reads.
//  * Bijective XCD-aware block remap: consecutive tiles (same A row panel) share an XCD L2.
#include "common.h"
#include "gemm_dev.h"

// RS_DIAG=1: the timing-diagnostic build (librescore_diag.so, build.py diag=True; tools/ only)
#ifndef RS_DIAG
#define RS_DIAG 0
#endif
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <type_traits>

namespace {

// LDS tile rows are BK fp16 = 2*BK bytes (BK = 64: 128 B, 8 chunks; BK = 32: 64 B, 4 chunks).
// Chunk swizzle spreading the 16 rows a ds_read_b128 lane group reads over the 16 slots of
// a 256-byte bank row: BK 64 -> chunk ^ ((row>>1)&7), BK 32 -> chunk ^ ((row>>2)&3).
template <int BK>
__device__ __forceinline__ int swz(int row, int chunk) {
    if constexpr (BK == 64) return chunk ^ ((row >> 1) & 7);
    else return chunk ^ ((row >> 2) & 3);
}



// MFMA shape abstraction: MS = 32 -> v_mfma_f32_32x32x16_f16 (16 accumulators per lane,
// 4 column quads), MS = 16 -> v_mfma_f32_16x16x32_f16 (4 accumulators, 1 quad).  Operands
// swapped (D = W_tile . A_tile^T): lane l owns output row (l % MS) of the block and, per quad
// g, the 4 consecutive columns qcol(g, l); fragment reads: lane l takes the 16 bytes of tile
// row (l % MS) at k-chunk (l / MS) of the substep (KPS = 512 / MS k per MFMA).
template <int MS> struct AccT;
template <> struct AccT<32> { typedef f32x16 type; };
template <> struct AccT<16> { typedef f32x4 type; };
template <int MS>
__device__ __forceinline__ typename AccT<MS>::type mfma_f16(half8 a, half8 b, typename AccT<MS>::type c) {
    if constexpr (MS == 32) return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    else return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
template <int MS>
__device__ __forceinline__ int qcol(int g, int lane) { return MS == 32 ? 8 * g + 4 * (lane >> 5) : 4 * (lane >> 4); }

// VAR bits: 128 (K loop software-pipelined by sched_group_barrier), 64 (non-temporal epilogue
// stores), 8192 (v_mfma_f32_16x16x32_f16).  (The measured-slower alternatives of rounds 1-3 —
// front-loaded reads, the direct permlane epilogue, the ping-pong wave rows, the two-buffer
// cross-step pipeline — are recorded in profiles/r1_*; their code was removed in round 4.)
template <int BM, int BN, int WM, int WN, int NSTAGE, int BK, int EPI, int VAR = 0>
__global__ void __launch_bounds__(WM * WN * 64)
gemm_f16_kernel(const f16* __restrict__ A, const f16* __restrict__ W, int K, int n_tiles_n,
                EpiArgs ep) {
    constexpr int NW = WM * WN;
    constexpr int A_BYTES = BM * BK * 2;
    constexpr int STAGE = (BM + BN) * BK * 2;
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int MS = (VAR & 8192) ? 16 : 32;         // MFMA shape (VAR bit 8192: 16x16x32)
    constexpr int KPS = 512 / MS, CPS = KPS / 8, NQ = MS * MS / 256;
    typedef typename AccT<MS>::type accT;
    constexpr int TM = WTM / MS, TN = WTN / MS;
    static_assert(MS == 32 || (EPI != EPI_LSE && BK / KPS >= 2), "16x16x32 MFMA: not the logsumexp epilogue");
    constexpr int RB = BK * 2;            // LDS row bytes
    constexpr int CPR = BK / 8;           // 16-byte chunks per row
    constexpr int RPP = 1024 / RB;        // rows per 1 KiB LDS-DMA piece
    constexpr int A_PIECES = BM / RPP, PIECES = (BM + BN) / RPP;
    static_assert(PIECES % NW == 0, "pieces per wave");
    constexpr int PPW = PIECES / NW;

    extern __shared__ __attribute__((aligned(16))) char smem[];

    // bijective XCD remap (blocks b and b+8 share an XCD on the observed dispatch)
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, pos = bid >> 3, q = nwg >> 3, r = nwg & 7;
    const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
    // grouped order: GM row panels x all column panels per group, column-major inside the
    // group, so the tiles an XCD runs together share weight panels in its L2
    int tm, tn;
    {
        const int GM = ep.group_m;
        const int n_tiles_m = nwg / n_tiles_n;
        const int per_group = GM * n_tiles_n;
        const int g = wgid / per_group, loc = wgid - g * per_group;
        const int gm = min(GM, n_tiles_m - g * GM);
        tn = loc / gm;
        tm = g * GM + (loc - tn * gm);
    }
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
        const int lrow = lane / CPR, pc = lane % CPR;
        if (piece < A_PIECES) {
            const int row = piece * RPP + lrow;
            src[p] = A + (size_t)(m0 + row) * K + swz<BK>(row, pc) * 8;
        } else {
            const int row = (piece - A_PIECES) * RPP + lrow;
            src[p] = W + (size_t)(n0 + row) * K + swz<BK>(row, pc) * 8;
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

    // Accumulators start at bias (+ residual): these loads' latency hides behind the whole
    // K loop and the epilogue only converts / activates / stores.
    //   acc[i][j][4g + e] <-> C[m0 + wm*WTM + MS*i + (lane%MS)][n0 + wn*WTN + MS*j + qcol(g) + e]
    accT acc[TM][TN];
    {
        const int arow = m0 + wm * WTM + (lane % MS);
        const int acol = n0 + wn * WTN;
        float2 rst[TM], rst0[TM];             // EPI_RESLN_F32: LN statistics of the residual rows
        const bool defer = EPI == EPI_RESLN_F32 && ep.res_o16 != nullptr;
        if constexpr (EPI == EPI_RESLN_F32) {
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                rst[i] = ep.res_stats[arow + MS * i];
                rst0[i] = defer ? ep.res_stats0[arow + MS * i] : make_float2(0.f, 0.f);
            }
        }
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int g = 0; g < NQ; ++g) {
                const int col = acol + MS * j + qcol<MS>(g, lane);
                const float4 b4 = *(const float4*)(ep.bias + col);
                float4 lg4, lb4, lg04, lb04;
                if constexpr (EPI == EPI_RESLN_F32) {
                    lg4 = *(const float4*)(ep.res_g + col);
                    lb4 = *(const float4*)(ep.res_b + col);
                    if (defer) {
                        lg04 = *(const float4*)(ep.res_g0 + col);
                        lb04 = *(const float4*)(ep.res_b0 + col);
                    }
                }
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    float4 v = b4;
                    if constexpr (EPI == EPI_RES_F32 || EPI == EPI_RESLN_F32) {
                        float4 r4 = *(const float4*)(ep.res + (size_t)(arow + MS * i) * ep.ldc + col);
                        if constexpr (EPI == EPI_RESLN_F32) {
                            if (defer) {   // post-attention stream: LN0(res) + o16 (ln_res_rows' x)
                                const half4 o = *(const half4*)(ep.res_o16 + (size_t)(arow + MS * i) * ep.ldc + col);
                                r4.x = ln_apply(r4.x, rst0[i], lg04.x, lb04.x) + (float)o[0];
                                r4.y = ln_apply(r4.y, rst0[i], lg04.y, lb04.y) + (float)o[1];
                                r4.z = ln_apply(r4.z, rst0[i], lg04.z, lb04.z) + (float)o[2];
                                r4.w = ln_apply(r4.w, rst0[i], lg04.w, lb04.w) + (float)o[3];
                            }
                            r4.x = ln_apply(r4.x, rst[i], lg4.x, lb4.x);
                            r4.y = ln_apply(r4.y, rst[i], lg4.y, lb4.y);
                            r4.z = ln_apply(r4.z, rst[i], lg4.z, lb4.z);
                            r4.w = ln_apply(r4.w, rst[i], lg4.w, lb4.w);
                        }
                        v = make_float4(v.x + r4.x, v.y + r4.y, v.z + r4.z, v.w + r4.w);
                    }
                    acc[i][j][4 * g] = v.x;
                    acc[i][j][4 * g + 1] = v.y;
                    acc[i][j][4 * g + 2] = v.z;
                    acc[i][j][4 * g + 3] = v.w;
                }
            }
    }

    const int nk = K / BK;
#pragma unroll
    for (int s = 0; s < NSTAGE - 1; ++s)
        if (s < nk) stage(s, s * BK);

    const int frow = lane % MS, fh = lane / MS;
    int buf = 0;
    for (int kt = 0; kt < nk; ++kt) {
        // tile kt landed for this wave: all later-issued stages may stay in flight
        {
            const int ahead = min(NSTAGE - 2, nk - 1 - kt);   // stages issued after tile kt
            if (NSTAGE >= 4 && ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPW) : "memory");
            else if (NSTAGE >= 3 && ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        // every wave's part of tile kt landed; every wave finished reading tile kt-1
        asm volatile("s_barrier" ::: "memory");
        int nb = buf + NSTAGE - 1;
        if (nb >= NSTAGE) nb -= NSTAGE;
        if (kt + NSTAGE - 1 < nk) stage(nb, (kt + NSTAGE - 1) * BK);
        if constexpr (VAR & 128) __builtin_amdgcn_sched_barrier(0);
        constexpr int NSUB = BK / KPS;         // k-substeps per stage
        const char* sA = smem + buf * STAGE;
        const char* sB = sA + A_BYTES;
        // fragments of k-substep s+1 are read while the MFMAs of substep s issue
        half8 af0[TM], bf0[TN], af1[TM], bf1[TN];
        auto load_frags = [&](int s, half8 (&af)[TM], half8 (&bf)[TN]) {
            const int lc = CPS * s + fh;
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int row = wn * WTN + j * MS + frow;
                bf[j] = *(const half8*)(sB + row * RB + (swz<BK>(row, lc) << 4));
            }
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int row = wm * WTM + i * MS + frow;
                af[i] = *(const half8*)(sA + row * RB + (swz<BK>(row, lc) << 4));
            }
        };
        auto mfmas = [&](const half8 (&af)[TM], const half8 (&bf)[TN]) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = mfma_f16<MS>(bf[j], af[i], acc[i][j]);
        };
        static_assert(NSUB == 2 || NSUB == 4, "substeps per stage");
        load_frags(0, af0, bf0);
        load_frags(1, af1, bf1);
        mfmas(af0, bf0);
        if constexpr (NSUB == 4) {
            load_frags(2, af0, bf0);
            mfmas(af1, bf1);
            load_frags(3, af1, bf1);
            mfmas(af0, bf0);
        }
        mfmas(af1, bf1);
        if constexpr ((VAR & 128) != 0) {
            // Software pipeline the scheduler will not find by itself (it serialises the
            // fragment reads and the MFMAs that consume them, exposing LDS latency per
            // substep): substep 0's reads, then substep s+1's reads one per MFMA of substep s.
            constexpr int NR = TM + TN, NM = TM * TN;
            static_assert(NM >= NR, "one read per MFMA slot");
            __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
#pragma unroll
            for (int s = 0; s < NSUB - 1; ++s) {
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                }
                __builtin_amdgcn_sched_group_barrier(0x008, NM - NR, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);
        }
        buf = buf + 1 == NSTAGE ? 0 : buf + 1;
    }
    // ---------------- epilogue.  acc[i][j][4g + e] = C[row][col + e],
    //   row = m0 + wm*WTM + 32i + (lane&31),  col = n0 + wn*WTN + 32j + 8g + 4(lane>>5)
    const int rbase = m0 + wm * WTM + frow;
    const int cbase = n0 + wn * WTN + 4 * fh;
    if constexpr (EPI == EPI_LSE) {
        static_assert(WTN == 64, "decoder logsumexp parts are 64-column slabs (n_parts = N/64)");
        // per (row, 64-column wave slab): max and sum exp over the slab + label logit
        const int slab = (n0 + wn * WTN) / WTN;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int row = rbase + i * 32;
            const int lab = row < ep.m_valid ? ep.label[row] : -1;
            float v[TN][16];
            float mx = -INFINITY;
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int col = cbase + j * 32 + 8 * g;

#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float x = col + e < ep.n_valid ? acc[i][j][4 * g + e] : -INFINITY;
                        v[j][4 * g + e] = x;
                        mx = fmaxf(mx, x);
                        if (col + e == lab) ep.label_logit[row] = x;
                    }
                }
            mx = fmaxf(mx, __shfl_xor(mx, 32));
            float sm = 0.f;
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) sm += v[j][e] == -INFINITY ? 0.f : __expf(v[j][e] - mx);
            sm += __shfl_xor(sm, 32);
            if (fh == 0 && row < ep.m_valid)
                ep.lse_part[(size_t)row * ep.n_parts + slab] = make_float2(mx, sm);
        }
    } else {
        // Through LDS: each wave parks one 32-row slice of its accumulators (fp32, row
        // stride WTN+4 floats: conflict-free b128 writes) in a private region, then reads it
        // back 8 consecutive columns per lane, so every global store covers whole 128/256-B
        // row segments instead of 16-B pieces of 32 rows.
        constexpr int LDW = WTN + 4;
        constexpr int LPR = WTN / 8, RPI = 64 / LPR, NIT = 32 / RPI;   // lanes/row, rows/pass
        static_assert(NW * 32 * LDW * 4 <= NSTAGE * STAGE, "epilogue LDS");
        __syncthreads();                                   // the LDS ring is no longer read
        float* lw = (float*)smem + wave * 32 * LDW;
        const int rr0 = lane / LPR, cc = (lane % LPR) * 8;
        const int col = n0 + wn * WTN + cc;
#pragma unroll
        for (int i32 = 0; i32 < WTM / 32; ++i32) {     // 32-row slices of the wave tile
#pragma unroll
            for (int sub = 0; sub < 32 / MS; ++sub) {
                const int i = i32 * (32 / MS) + sub;
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int g = 0; g < NQ; ++g)
                        *(float4*)(lw + (sub * MS + frow) * LDW + j * MS + qcol<MS>(g, lane)) =
                            make_float4(acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
            }
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                const int rr = it * RPI + rr0;
                const int row = m0 + wm * WTM + i32 * 32 + rr;
                const float4 u0 = *(const float4*)(lw + rr * LDW + cc);
                const float4 u1 = *(const float4*)(lw + rr * LDW + cc + 4);
                float x[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
                if (row < ep.m_valid) {
                    const size_t o = (size_t)row * ep.ldc + col;
                    if constexpr (EPI == EPI_GELU_F16 || EPI == EPI_GELU_F32) {
#pragma unroll
                        for (int e = 0; e < 8; e += 2) {
                            const f32x2 gv = gelu2((f32x2){x[e], x[e + 1]});
                            x[e] = gv.x;
                            x[e + 1] = gv.y;
                        }
                    }
                    if constexpr (EPI == EPI_BIAS_F16) {
                        half8 h;
#pragma unroll
                        for (int e = 0; e < 8; ++e) h[e] = (f16)x[e];
                        st16<VAR>((uint4*)((f16*)ep.out + o), __builtin_bit_cast(uint4, h));
                    } else if constexpr (EPI == EPI_GELU_F16) {
                        f16* orow = (f16*)ep.out + (size_t)row * ep.ldc;
                        half8 h, l, md;
#pragma unroll
                        for (int e = 0; e < 8; ++e) {
                            h[e] = (f16)x[e];
                            l[e] = x3_lo(x[e], h[e]);
                            md[e] = x3_mid(h[e]);
                        }
                        st16<VAR>((uint4*)(orow + col), __builtin_bit_cast(uint4, h));
                        if (ep.kx == 3) {
                            st16<VAR>((uint4*)(orow + ep.nlog + col), __builtin_bit_cast(uint4, md));
                            st16<VAR>((uint4*)(orow + 2 * ep.nlog + col), __builtin_bit_cast(uint4, l));
                        }
                    } else {  // fp32 outputs (residual already in acc)
                        st16<VAR>((uint4*)((float*)ep.out + o), __builtin_bit_cast(uint4, make_float4(x[0], x[1], x[2], x[3])));
                        st16<VAR>((uint4*)((float*)ep.out + o + 4), __builtin_bit_cast(uint4, make_float4(x[4], x[5], x[6], x[7])));
                    }
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------------------
// Persistent variant for the fp16-output epilogues (fused QKV, BertIntermediate) in the
// fp16 precision mode (kx = 1).  256x256 tiles, 8 waves (2x4), BK 64, two LDS buffers and
// the software-pipelined K loop of gemm_f16_kernel; one workgroup per CU walks the tiles
// t = blockIdx.x, + gridDim.x, ... (gridDim.x a multiple of 8, so a tile keeps the XCD its
// block runs on and the same bijective XCD remap applies to t).
// Per tile transition: barrier -> the NEXT tile's stage 0 (buffer 0) and bias are issued ->
// this tile's epilogue (bias/GELU applied in registers, fp16, transposed through a per-wave
// slab in buffer 1, whole 128-B row segments stored non-temporally).  The next tile then
// waits vmcnt(NSTORE): its stage 0 and bias, not the stores (the stores are unconditional,
// rows < M_pad are all allocated, so NSTORE is exact).  The bias loads are inline asm so the
// compiler's own (loop-merged, conservative) wait does not drain the stores; the wait asm
// takes the bias registers as operands, so nothing reads them before it.
template <int EPI, int VAR>
__global__ void __launch_bounds__(512)
gemm_persist_kernel(const f16* __restrict__ A, const f16* __restrict__ W, int K, int n_tiles_n,
                    int n_tiles, EpiArgs ep) {
    constexpr int BM = 256, BN = 256, WN = 4, BK = 64, NW = 8;
    constexpr int A_BYTES = BM * BK * 2, STAGE = (BM + BN) * BK * 2;
    constexpr int WTM = 128, WTN = 64;
    constexpr int MS = 32;                        // v_mfma_f32_32x32x16_f16 (16x16: +7 % QKV time)
    constexpr int KPS = 512 / MS, CPS = KPS / 8, NQ = MS * MS / 256;
    typedef typename AccT<MS>::type accT;
    constexpr int TM = WTM / MS, TN = WTN / MS, NBQ = TN * NQ;   // NBQ: bias quads per lane
    constexpr int RB = BK * 2, CPR = BK / 8, RPP = 1024 / RB;
    constexpr int A_PIECES = BM / RPP, PIECES = (BM + BN) / RPP, PPW = PIECES / NW;
    constexpr int NSTORE = (WTM / 32) * 4;        // 16-B stores per wave per tile
    constexpr int NSUB = BK / KPS, NR = TM + TN, NM = TM * TN;
    static_assert(EPI == EPI_BIAS_F16 || EPI == EPI_GELU_F16, "fp16-output epilogues only");
    // VAR 4194304: fp16x3 precision mode (kx = 3) — the GELU output is written as the
    // three-part operand image [hi | hi/64 | lo·64] of the next GEMM (ep.nlog columns apart)
    constexpr bool X3 = (VAR & 4194304) != 0;
    static_assert(!X3 || EPI == EPI_GELU_F16, "x3 image: GELU");
    static_assert(NW * 32 * 128 <= STAGE, "epilogue slab fits in one buffer");
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;
    const int frow = lane % MS, fh = lane / MS;
    const int nk = K / BK;

    int t = blockIdx.x;
    if (t >= n_tiles) return;
    // VAR 262144: static priority for the second-dispatched wave half (MI355X_MICROARCH
    // 'Two waves per SIMD' item 4: the younger wave of each SIMD loses every arbitration)
    if constexpr ((VAR & 262144) != 0) {
        if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
    }
    auto tile_of = [&](int tt, int& m0, int& n0) {
        const int xcd = tt & 7, pos = tt >> 3, q = n_tiles >> 3, r = n_tiles & 7;
        const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
        const int GM = ep.group_m, n_tiles_m = n_tiles / n_tiles_n, per_group = GM * n_tiles_n;
        const int g = wgid / per_group, loc = wgid - g * per_group;
        const int gm = min(GM, n_tiles_m - g * GM);
        const int tn = loc / gm;
        m0 = (g * GM + (loc - tn * gm)) * BM;
        n0 = tn * BN;
    };
    // Pieces p < 4 of a wave are A rows (p*8 + wave)*8 + lane/8, pieces p >= 4 the same rows
    // of W: 64 rows apart with a p-independent swizzle ((row>>1)&7 depends on wave and lane
    // only), so two per-lane bases and a scalar stride address all eight.
    static_assert(A_PIECES == 4 * NW && PIECES == 8 * NW && RPP == 8, "piece layout");
    const int lrow = lane / CPR, pc = lane % CPR;
    const int prow = wave * RPP + lrow;                 // row of piece 0 (and of piece 4 in W)
    const int pswz = swz<BK>(prow, pc) * 8;
    const size_t pstride = (size_t)64 * K;              // elements between pieces p and p+1
    const f16* srcA;
    const f16* srcW;
    auto set_src = [&](int m0, int n0) {
        srcA = A + (size_t)(m0 + prow) * K + pswz;
        srcW = W + (size_t)(n0 + prow) * K + pswz;
    };
    auto stage = [&](int buf, int k0) {
#pragma unroll
        for (int p = 0; p < PPW; ++p) {
            const f16* g = (p < 4 ? srcA + p * pstride : srcW + (p - 4) * pstride) + k0;
            __builtin_amdgcn_global_load_lds((const void*)g,
                                             (__attribute__((address_space(3))) void*)(smem + buf * STAGE + (p * NW + wave) * 1024),
                                             16, 0, 0);
        }
    };
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    f32x4 bz[NBQ];                                // bias of the tile about to start (quad j*NQ+g)
    auto load_bias = [&](int n0) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int g = 0; g < NQ; ++g) {
                const float* bp = ep.bias + n0 + wn * WTN + MS * j + qcol<MS>(g, lane);
                asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(bz[j * NQ + g]) : "v"(bp) : "memory");
            }
    };
    static_assert(NBQ == 8 || NBQ == 4, "RS_PERSIST_WAIT operand list");
#define RS_PERSIST_WAIT(N)                                                                         \
    if constexpr (NBQ == 8)                                                                        \
        asm volatile("s_waitcnt vmcnt(" #N ")"                                                     \
                     : "+v"(bz[0]), "+v"(bz[1]), "+v"(bz[2]), "+v"(bz[3]), "+v"(bz[4]), "+v"(bz[5]), \
                       "+v"(bz[6]), "+v"(bz[7])                                                     \
                     :                                                                              \
                     : "memory");                                                                   \
    else                                                                                            \
        asm volatile("s_waitcnt vmcnt(" #N ")"                                                     \
                     : "+v"(bz[0]), "+v"(bz[1]), "+v"(bz[2]), "+v"(bz[3])                           \
                     :                                                                              \
                     : "memory")

    int m0, n0;
    tile_of(t, m0, n0);
    set_src(m0, n0);
    stage(0, 0);
    load_bias(n0);
    RS_PERSIST_WAIT(0);
    const int offA = (wm * WTM + frow) * RB + (swz<BK>(wm * WTM + frow, fh) << 4);
    const int offB = A_BYTES + (wn * WTN + frow) * RB + (swz<BK>(wn * WTN + frow, fh) << 4);
    for (;;) {
        accT acc[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int g = 0; g < NQ; ++g) {
                    acc[i][j][4 * g] = bz[j * NQ + g].x;
                    acc[i][j][4 * g + 1] = bz[j * NQ + g].y;
                    acc[i][j][4 * g + 2] = bz[j * NQ + g].z;
                    acc[i][j][4 * g + 3] = bz[j * NQ + g].w;
                }
        // ---- K loop: stage kt landed (this tile's stage 0 was waited with the bias).  STAG:
        // this wave runs the staggered schedule (VAR 524288, younger half); one loop body per
        // schedule, chosen once per tile, so each is register-allocated on its own.
        auto kloop = [&](auto stag_tag) {
        constexpr bool STAG = decltype(stag_tag)::value;
        half8 af0[TM], bf0[TN], af1[TM], bf1[TN];   // (staggered waves carry af1/bf1 across steps)
        for (int kt = 0; kt < nk; ++kt) {
            if (kt > 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("s_barrier" ::: "memory");
            if (kt + 1 < nk) stage((kt + 1) & 1, (kt + 1) * BK);
            __builtin_amdgcn_sched_barrier(0);
            const char* sb = smem + (kt & 1) * STAGE;
            // substep s covers chunks CPS*s .. CPS*s + CPS-1: one XOR of the per-lane base
            auto load_frags = [&](int s, half8 (&af)[TM], half8 (&bf)[TN]) {
                const int xa = offA ^ ((CPS * s) << 4), xb = offB ^ ((CPS * s) << 4);
#pragma unroll
                for (int j = 0; j < TN; ++j) bf[j] = *(const half8*)(sb + xb + j * MS * RB);
#pragma unroll
                for (int i = 0; i < TM; ++i) af[i] = *(const half8*)(sb + xa + i * MS * RB);
            };
            auto mfmas = [&](const half8 (&af)[TM], const half8 (&bf)[TN]) {
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = mfma_f16<MS>(bf[j], af[i], acc[i][j]);
            };
            static_assert(NSUB == 2 || NSUB == 4, "substeps per K-step");
            if constexpr (NSUB == 4 && STAG) {
                {
                    // Stagger (MI355X_MICROARCH 'Two waves per SIMD' item 9): the younger wave
                    // half runs one substep behind — its last substep's MFMAs (fragments already
                    // in af1/bf1, read before this K-step's barrier) issue after the barrier,
                    // beside the next K-step's substep-0 reads, so the two waves of a SIMD do not
                    // reach their MFMA bursts and LDS read bursts in lockstep.
                    if (kt > 0) {
                        mfmas(af1, bf1);
                        load_frags(0, af0, bf0);
#pragma unroll
                        for (int r = 0; r < NR; ++r) {
                            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                        }
                        __builtin_amdgcn_sched_group_barrier(0x008, NM - NR, 0);
                    } else {
                        load_frags(0, af0, bf0);
                        __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    load_frags(1, af1, bf1);
                    mfmas(af0, bf0);
                    load_frags(2, af0, bf0);
                    mfmas(af1, bf1);
                    load_frags(3, af1, bf1);
                    mfmas(af0, bf0);
#pragma unroll
                    for (int q = 0; q < 3; ++q) {
#pragma unroll
                        for (int r = 0; r < NR; ++r) {
                            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                        }
                        __builtin_amdgcn_sched_group_barrier(0x008, NM - NR, 0);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    if (kt + 1 == nk) {
                        mfmas(af1, bf1);          // the deferred last substep of the tile
                    } else {
                        // WAR: the deferred fragments are read from the buffer the next K-step
                        // refills after its barrier — retire those reads before reaching it
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    }
                    continue;
                }
            }
            load_frags(0, af0, bf0);
            load_frags(1, af1, bf1);
            mfmas(af0, bf0);
            if constexpr (NSUB == 4) {
                load_frags(2, af0, bf0);
                mfmas(af1, bf1);
                load_frags(3, af1, bf1);
                mfmas(af0, bf0);
            }
            mfmas(af1, bf1);
            __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
#pragma unroll
            for (int s = 0; s < NSUB - 1; ++s) {
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                }
                __builtin_amdgcn_sched_group_barrier(0x008, NM - NR, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, NM, 0);
        }
        };
        if constexpr (NSUB == 4 && (VAR & 524288) != 0) {
            if (wave >= NW / 2) kloop(std::true_type{});
            else kloop(std::false_type{});
        } else {
            kloop(std::false_type{});
        }
        // ---- transition: next tile's stage 0 + bias, then this tile's epilogue
        // every wave is done reading the ring (the slab lives in buffer 1).  VAR 1048576: the
        // slabs have their own LDS, and with an even K-step count the next tile's stage 0
        // (buffer 0) was last read before the final K-step's barrier, so no wave waits here
        if (!(VAR & 1048576) || (nk & 1)) asm volatile("s_barrier" ::: "memory");
        const int cm0 = m0, cn0 = n0;
        bool more = false;
        auto issue_next = [&]() {
            t += gridDim.x;
            more = t < n_tiles;
            if (more) {
                tile_of(t, m0, n0);
                set_src(m0, n0);
                stage(0, 0);     // buffer 0: free (barrier above, or last read before the final K-step's)
                load_bias(n0);
            }
        };
        // epilogue part 1: bias/GELU, fp16, transposed through the wave's slab (buffer 1) into
        // whole-row registers; no LDS access follows the next tile's DMA issue below
        const int rr0 = lane >> 3, cc = (lane & 7) * 8;
        uint4 ov[WTM / 32][4];
        f16* obase = (f16*)ep.out + (size_t)(cm0 + wm * WTM + rr0) * ep.ldc + cn0 + wn * WTN + cc;
        {
            // 32x32x16 accumulators: v_permlane32_swap packs 8 consecutive columns per lane
            // (lanes 0-31 the low, 32-63 the high 8 of each 16-column pair), stored as one
            // ds_write_b128 into 128-B slab rows with the 16-B chunk XOR-swizzled by (row & 7):
            // the 8-lane write groups (8 rows, one chunk) and the 16-lane read groups (two rows,
            // all chunks) are both conflict-free (a padded layout measured 2-way on both, round 1)
            static_assert(WTN == 64, "slab rows of 8 chunks");
            char* slb = smem + ((VAR & 1048576) ? 2 * STAGE : STAGE) + wave * 32 * 128;
            if constexpr (X3) {
                // fp16x3 image [hi | hi/64 | lo·64] (common.h put_split): GELU once, in place
#pragma unroll
                for (int i32 = 0; i32 < WTM / 32; ++i32)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
#pragma unroll
                        for (int e = 0; e < 16; e += 2) {
                            const f32x2 gv = gelu2((f32x2){acc[i32][j][e], acc[i32][j][e + 1]});
                            acc[i32][j][e] = gv.x;
                            acc[i32][j][e + 1] = gv.y;
                        }
            }
            // image img (0: hi, 1: hi/64, 2: lo·64) of the tile through the slab into ov;
            // STORE_NOW: each 32-row slice is stored as soon as it is read back (images 0/1:
            // only 16 registers of ov live beside the 128 accumulators)
            auto build_img = [&](int img, auto store_now) {
                constexpr bool STORE_NOW = decltype(store_now)::value;
#pragma unroll
            for (int i32 = 0; i32 < WTM / 32; ++i32) {
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int gp = 0; gp < 2; ++gp) {
                        float x[8];
#pragma unroll
                        for (int e = 0; e < 8; ++e) x[e] = acc[i32][j][8 * gp + e];
                        if constexpr (EPI == EPI_GELU_F16 && !X3) {
#pragma unroll
                            for (int e = 0; e < 8; e += 2) {
                                const f32x2 gv = gelu2((f32x2){x[e], x[e + 1]});
                                x[e] = gv.x;
                                x[e + 1] = gv.y;
                            }
                        }
                        half8 h;
#pragma unroll
                        for (int e = 0; e < 8; ++e) h[e] = (f16)x[e];
                        if constexpr (X3) {
                            if (img == 1) {
#pragma unroll
                                for (int e = 0; e < 8; ++e) h[e] = x3_mid(h[e]);
                            } else if (img == 2) {
#pragma unroll
                                for (int e = 0; e < 8; ++e) h[e] = x3_lo(x[e], h[e]);
                            }
                        }
                        const uint4 hv = __builtin_bit_cast(uint4, h);   // .xy group 2gp, .zw group 2gp+1
                        const auto s0 = __builtin_amdgcn_permlane32_swap(hv.x, hv.z, false, false);
                        const auto s1 = __builtin_amdgcn_permlane32_swap(hv.y, hv.w, false, false);
                        const int c = 4 * j + 2 * gp + fh;               // 16-B chunk of the row
                        *(uint4*)(slb + frow * 128 + ((c ^ (frow & 7)) << 4)) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
                    }
#pragma unroll
                for (int it = 0; it < 4; ++it)
                    ov[STORE_NOW ? 0 : i32][it] = *(const uint4*)(slb + (it * 8 + rr0) * 128 + (((lane & 7) ^ rr0) << 4));
                if constexpr (STORE_NOW) {
#pragma unroll
                    for (int it = 0; it < 4; ++it)
                        st16<64>((uint4*)(obase + img * ep.nlog + (size_t)(i32 * 32 + it * 8) * ep.ldc), ov[0][it]);
                }
            }
            };
            if constexpr (X3) {
                // images 0 and 1 are stored before the next tile's DMA issue (the slab is
                // wave-private: LDS ops of a wave run in order, so the rewrite after the reads
                // is safe); image 2 takes the overlapped store slot below
                build_img(0, std::true_type{});
                build_img(1, std::true_type{});
                build_img(2, std::false_type{});
                obase += 2 * ep.nlog;
            } else {
                build_img(0, std::false_type{});
            }
        }
        // part 2: the next tile's stage 0 (buffer 0) and bias
        issue_next();
        // part 3: this tile's stores (whole 128-B row segments, non-temporal)
#pragma unroll
        for (int i = 0; i < WTM / 32; ++i)
#pragma unroll
            for (int it = 0; it < 4; ++it)
                st16<64>((uint4*)(obase + (size_t)(i * 32 + it * 8) * ep.ldc), ov[i][it]);
        if (!more) break;
        RS_PERSIST_WAIT(16);
        static_assert(NSTORE == 16, "RS_PERSIST_WAIT count");
    }
#undef RS_PERSIST_WAIT
}



// ---------------------------------------------------------------------------------------
// fp16x3 with SPLIT operands ("x3s"): the fp32-accurate product A . W^T as three fp16 MFMA
// products from two-part images, A = [A_hi | A_lo*64] ([M, 2K]) and W = [W_hi | W_lo*64]
// ([N, 2K]) (common.h put_split2):
//     acc += W_hi . A_hi  +  (W_hi/64) . (A_lo*64)  +  (W_lo*64) . (A_hi/64)
// the /64 factors applied to the fragments in registers (v_pk_mul_f16; the power-of-two
// factors cancel exactly, the MFMA's subnormal flush drops the same terms the three-part
// images of the K-concatenated form drop).  Against that form (K x 3 over [hi | hi/64 | lo*64]
// images) every LDS-DMA byte and every fragment read feeds 1.5x the MFMA work: a K-step of
// BK = 32 stages A_hi, A_lo, W_hi, W_lo (4 x 16 KiB, the same 64 KiB stage) for 3 products.
// Persistent: one workgroup per CU walks 256x256 tiles (8 waves, 128x64 each, 32x32x16 MFMA),
// two LDS stages, one barrier per K-step, after which step kt+1's DMA goes into the buffer
// step kt-1 used (one K-step of lead).  One fragment set per wave (the two-set software
// pipeline does not fit 2 waves/SIMD: 128 accumulators + 2 x 48 fragment registers); the
// partner wave of the SIMD covers a wave's read latency.  Tile transition: the next tile's
// stage 0 goes into the free buffer before this tile's epilogue, so the next tile's first
// wait leaves this tile's stores in flight.
// Epilogues: EPI_BIAS_F32 (fp32 [M, ldc]), EPI_GELU_F16 (two-part GELU image, nlog apart),
// EPI_BIAS_F16; bias added in the epilogue (its loads ride the last K-step).  Rows up to
// M_pad are stored (the buffers are M_pad rows).
// ---- LayerNorm-epilogue gangs: first-tile tickets (thread 0 of a workgroup) -------------------
// Counter words of ep.lncnt (zeroed once by the owner; the last workgroup to finish a launch zeroes
// them again, lnr_done, so each launch on the stream starts from zero — no host-side ticket state):
enum : int {
    LNC_DONE = 16,         // workgroups finished
    LNC_LOCAL = 32,        // + 16 x: XCD x's local ticket (own 64-B line each)
    LNC_OVF = 176,         // overflow ticket (every gang of RS_LNGANG=ticket)
    LNC_GANGS = 192,       // panel lists taken
    LNC_WORDS = 256,
    LNC_TAB = 128,         // u64 index of the gang slots {ln_tag, state}: [8][128] local, then [256] overflow
    LNC_TAB_N = 8 * 128 + 256,
};
constexpr size_t lnr_counter_bytes() { return (size_t)LNC_TAB * 8 + (size_t)LNC_TAB_N * 8; }

// Bounds of the waits in a LayerNorm-GEMM launch, in ticks of the constant 100 MHz s_memrealtime
// clock.  Statistics (between members of a formed gang, which have all started): 1 s.  Gang
// formation (a member waiting for workgroups that have not started — under another tenant's
// kernels they start when a CU frees up in their shader engine): 10 s, a hang guard only.
// RS_LNFUSE_DIAG=8 (tests): 10 us.  A wait that runs out sets the sticky error word; every other
// wait that sees it gives up, so the launch drains and the call returns RS_EHIP.
__device__ __forceinline__ unsigned long long lnr_wait_ticks(int diag) { return (diag & 8) ? 1000ull : 100000000ull; }
__device__ __forceinline__ unsigned long long lnr_form_ticks(int diag) { return (diag & 8) ? 1000ull : 1000000000ull; }
__device__ __forceinline__ unsigned long long lnr_now() { return __builtin_amdgcn_s_memrealtime(); }

typedef __attribute__((address_space(1))) unsigned lgu32;
typedef __attribute__((address_space(1))) unsigned long long lgu64;
__device__ __forceinline__ unsigned lnr_add(unsigned* c, int w, unsigned v = 1u) {
    return __hip_atomic_fetch_add((lgu32*)(c + w), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned lnr_ld(const unsigned* c, int w) {
    return __hip_atomic_load((const lgu32*)(c + w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Gangs (thread 0 of every workgroup, once at its start).  A gang = the ntn workgroups computing
// the column tiles of the same row panels, formed only from workgroups that have STARTED (the
// hardware dispatches a grid's workgroups round-robin over the 32 shader engines, and one whose
// engine is full waits there however many CUs are free elsewhere: blockIdx says nothing about
// co-residency).  XCD (RS_LNGANG=xcd): gangs inside one XCD (its column tiles then read their
// shared A panel through one L2) — XCD x's workgroups take local tickets in start order, and every
// ntn consecutive local tickets below cap = floor(floor(G / 8) / ntn) * ntn form a local gang.
// Otherwise, and for the local tickets past cap and the members of cancelled local gangs: gangs of
// ntn consecutive overflow tickets, in start order.  A gang is settled exactly once in its slot
// {ln_tag, state} by compare-and-swap: its completing member claims it (PENDING), takes the next
// panel list and publishes its id; a waiting member cancels it instead when every list has been
// taken (no work is left for it), or, for a local gang, after LNR_CANCEL_TICKS (its XCD has fewer
// than ntn free slots: the members regroup chip-wide).  Whoever wins decides for every member,
// present or arriving later.  Panel lists: list l of NL = min(G / ntn, panels) holds the row panels
// l, l + G / ntn, ...; a gang walks its list (member m keeps column tile m), then takes the next
// untaken list (lnr: the list counter; in the normal case none is left, every gang having formed
// with its own), so the lists of gangs that never formed — workgroups held off by another tenant
// — are computed by the gangs that did, and nothing waits for a workgroup that has not started.
// Returns l * ntn + m (l >= NL: no work) or ~0u after a timeout (the launch drains).
constexpr unsigned LNR_PENDING = 0xfffffffeu, LNR_CANCELLED = 0xffffffffu;
constexpr unsigned long long LNR_CANCEL_TICKS = 5000ull;      // 50 us of the 100 MHz clock
template <bool XCD>
__device__ unsigned lnr_gang_ticket(const EpiArgs& ep, int ntn_, int n_panels) {
    unsigned* c = ep.lncnt;
    const unsigned ntn = (unsigned)ntn_, G = gridDim.x;
    const unsigned long long tag = (unsigned long long)ep.ln_tag << 32;
    unsigned long long* tab = (unsigned long long*)c + LNC_TAB;
    const unsigned long long t_lim = lnr_form_ticks(ep.diag), t_start = lnr_now();
    auto ld64 = [](unsigned long long* p) {
        return __hip_atomic_load((const lgu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    auto cas64 = [](unsigned long long* p, unsigned long long& expect, unsigned long long want) {
        return __hip_atomic_compare_exchange_strong((lgu64*)p, &expect, want, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
    };
    const unsigned NL = min(G / ntn, (unsigned)n_panels);
    auto exhausted = [&]() { return lnr_ld(c, LNC_GANGS) >= NL; };
    // the completing member: claim the slot (unless cancelled), take a panel list, publish its id
    auto complete = [&](unsigned long long* slot, unsigned& gid) -> bool {
        unsigned long long v = ld64(slot);
        for (;;) {
            if ((v >> 32) == (tag >> 32)) return false;                // cancelled (no one else claims)
            if (cas64(slot, v, tag | LNR_PENDING)) break;
        }
        gid = lnr_add(c, LNC_GANGS);
        __hip_atomic_store((lgu64*)slot, tag | gid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return true;
    };
    // a waiting member: 1 published (gid), -1 cancelled, 0 timed out / the error word set
    auto await_id = [&](unsigned long long* slot, bool local, unsigned& gid) -> int {
        const unsigned long long t0 = lnr_now();
        for (unsigned spins = 1;; ++spins) {
            unsigned long long v = ld64(slot);
            if ((v >> 32) == (tag >> 32)) {
                const unsigned st = (unsigned)v;
                if (st == LNR_CANCELLED) return -1;
                if (st != LNR_PENDING) {
                    gid = st;
                    return 1;
                }
            } else if ((local && lnr_now() - t0 > ((ep.diag & 8) ? 0ull : LNR_CANCEL_TICKS)) || exhausted()) {
                if (cas64(slot, v, tag | LNR_CANCELLED)) return -1;
                continue;                                          // settled meanwhile: read it again
            }
            if ((spins & 63) == 0 && (lnr_now() - t_start > t_lim || lnr_ld(ep.lnerr, 0))) return 0;
            __builtin_amdgcn_s_sleep(1);
        }
    };
    unsigned gid = 0, mem = 0;
    bool ovf = !XCD, ok = true;
    if constexpr (XCD) {
        unsigned x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
        x &= 7;
        const unsigned cap = (G / 8) / ntn * ntn;
        const unsigned lc = lnr_add(c, LNC_LOCAL + 16 * (int)x);
        ovf = lc >= cap;
        if (!ovf) {
            const unsigned k = lc / ntn;
            mem = lc - k * ntn;
            unsigned long long* slot = tab + x * 128 + k;
            if (mem + 1 == ntn) {
                ovf = !complete(slot, gid);
            } else {
                const int r = await_id(slot, true, gid);
                ok = r != 0;
                ovf = r < 0;
            }
        }
    }
    if (ovf && ok) {
        const unsigned o = lnr_add(c, LNC_OVF), k = o / ntn;
        mem = o - k * ntn;
        unsigned long long* slot = tab + 8 * 128 + k;
        if (k >= 256) {
            ok = false;
        } else if (mem + 1 == ntn) {
            if (!complete(slot, gid)) gid = NL;                        // cancelled: no work left
        } else {
            const int r = await_id(slot, false, gid);
            ok = r != 0;
            if (r < 0) gid = NL;
        }
    }
    if (!ok) {
        __hip_atomic_store((lgu32*)ep.lnerr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0xffffffffu;
    }
    return gid >= NL ? 0xfffffffeu : gid * ntn + mem;
}

// The transition after the last tile of a gang's panel list (panel p, column tile tcol): column tile
// 0's wave 0 publishes the list it took (nlist, its lane 0) in the claim granule of panel p, after
// the launch's statistics granules; every wave of every member reads it there.  t = the new list's
// first tile, or past the tiles.  false: the wait ran out or the error word is set (the launch
// drains; the sticky word is set).
__device__ __forceinline__ bool lnr_next_list(const EpiArgs& ep, int& t, unsigned nlist, int p, int tcol, int ntn,
                                              int n_tiles, int wave, int lane) {
    const int n_panels = n_tiles / ntn;
    const unsigned NL = min((unsigned)(gridDim.x / ntn), (unsigned)n_panels);
    const unsigned long long tag = (unsigned long long)ep.ln_tag << 32;
    unsigned long long* clm = (unsigned long long*)ep.lnx + (size_t)n_panels * ntn * 512 + p;
    if (tcol == 0 && wave == 0 && lane == 0)
        __hip_atomic_store((lgu64*)clm, tag | nlist, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long t_lim = lnr_wait_ticks(ep.diag), t_start = lnr_now();
    for (unsigned spins = 1;; ++spins) {
        const unsigned long long v = __hip_atomic_load((const lgu64*)clm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((v >> 32) == (tag >> 32) && !(ep.diag & 8)) {
            const unsigned l = (unsigned)v;
            t = l < NL ? (int)l * ntn + tcol : n_tiles;
            return true;
        }
        if ((spins & 63) == 0 && (lnr_now() - t_start > t_lim || lnr_ld(ep.lnerr, 0))) {
            if (lane == 0) __hip_atomic_store((lgu32*)ep.lnerr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// End of a workgroup (thread 0): the last of the grid zeroes the counters for the next launch
// (every workgroup has taken its tickets by then: each adds to LNC_DONE after its own).
__device__ __forceinline__ void lnr_done(const EpiArgs& ep) {
    unsigned* c = ep.lncnt;
    if (lnr_add(c, LNC_DONE) + 1 != gridDim.x) return;
    const int w[] = {LNC_OVF, LNC_GANGS, LNC_DONE};
    for (int x = 0; x < 8; ++x) __hip_atomic_store((lgu32*)(c + LNC_LOCAL + 16 * x), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int i = 0; i < 3; ++i) __hip_atomic_store((lgu32*)(c + w[i]), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int EPI, int VAR>
__global__ void __launch_bounds__(512)
gemm_x3s_kernel(const f16* __restrict__ A, const f16* __restrict__ W, int K, int ldw, int n_tiles_n, int n_tiles,
                EpiArgs ep) {
    constexpr int BM = 256, BK = 32, NW = 8, WN = 4, WTM = 128, WTN = 64;
    constexpr int RB = BK * 2;                   // 64-byte LDS rows
    constexpr int REG = BM * RB;                 // one 256-row region: 16 KiB
    constexpr int STAGE = 4 * REG;               // A_hi | A_lo | W_hi | W_lo
    constexpr int NSTORE = 32;                   // epilogue stores per wave per tile
    static_assert(EPI == EPI_BIAS_F32 || EPI == EPI_GELU_F16 || EPI == EPI_LNRES_IMG, "x3s epilogues");
    constexpr bool LNR = EPI == EPI_LNRES_IMG;
    // Timing diagnostics (wrong results; compiled only into the RS_DIAG build, librescore_diag.so,
    // never into the shipped library): DV 1 no K-loop staging, 2 no epilogue stores, 8 the DMA
    // never waited for, 33554432 every tile stores onto row panel 0 (no HBM write burst),
    // 268435456 the stamp build (rs_debug_stamps): s_memtime at the tile's phase boundaries,
    // per-phase cycle sums in scalar registers, stored by thread 0 into
    // ep.dbg[blockIdx.x * 16 + phase] (a buffer of its own: no output depends on it)
    constexpr int DV = RS_DIAG ? VAR & (1 | 2 | 8 | 33554432 | 268435456) : 0;
    static_assert(!LNR || (DV & 2) == 0, "the LayerNorm epilogue has no no-store diagnostic");
    constexpr bool STAMP = (DV & 268435456) != 0;
    unsigned long long st_sum[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, st_prev = 0;
    auto stamp = [&](int ph) __attribute__((always_inline)) {
        if constexpr (STAMP) {
            unsigned long long tt;
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tt)::"memory");
            __builtin_amdgcn_sched_barrier(0);
            if (ph >= 0) st_sum[ph] += tt - st_prev;
            st_prev = tt;
        }
    };
    stamp(-1);
    static_assert((VAR & 16777216) == 0 || LNR, "the permuted-column layout is written for the LayerNorm epilogue");
    extern __shared__ __attribute__((aligned(16))) char smem[];        // the LDS-DMA ring (2 stages)
    // wave-private epilogue slabs: a separate LDS object, so the compiler can tell the slab
    // reads do not alias the LDS-DMA writes in flight (no vmcnt wait before them)
    __shared__ __attribute__((aligned(16))) char slabs[NW * 4096];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN, wn = wave % WN;
    const int nk = K / BK;
    int t = blockIdx.x;
    typedef __attribute__((address_space(1))) unsigned gu32;
    typedef __attribute__((address_space(1))) unsigned long long gu64;
    if constexpr (LNR) {
        // Gangs: a row panel's n_tiles_n column tiles are computed by n_tiles_n workgroups that
        // exchange row statistics (lnres_epilogue), so a gang must consist of workgroups that have
        // all STARTED: gangs are formed from tickets taken at start, never from blockIdx.  A gang
        // walks panel list l (panels l, l + G / ntn, ...; member m keeps column tile m: first tile
        // l * ntn + m, then t += gridDim.x), then the next untaken list.  lnr_gang_ticket (thread 0)
        // returns l * ntn + m.
        if (tid == 0) *(unsigned*)(slabs + 2048) = lnr_gang_ticket<(VAR & 134217728) != 0>(ep, n_tiles_n, n_tiles / n_tiles_n);
        __syncthreads();
        t = (int)*(const unsigned*)(slabs + 2048);
    }
    stamp(8);
    if ((unsigned)t >= (unsigned)n_tiles) {
        if constexpr (LNR) {
            if (tid == 0) lnr_done(ep);
        }
        return;
    }
    if ((unsigned)t >= (unsigned)n_tiles) return;
    // the younger wave half (waves 4-7, one per SIMD beside an older partner) at s_setprio 1
    // (MI355X_MICROARCH 'Two waves per SIMD' item 4)
    if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
    auto tile_of = [&](int tt, int& m0, int& n0) {
        if constexpr (LNR) {                      // row panel t / ntn, column tile t % ntn
            m0 = (tt / n_tiles_n) * BM;
            n0 = (tt - (tt / n_tiles_n) * n_tiles_n) * BM;
            return;
        }
        const int xcd = tt & 7, pos = tt >> 3, q = n_tiles >> 3, r = n_tiles & 7;
        const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
        const int GM = ep.group_m, n_tiles_m = n_tiles / n_tiles_n, per_group = GM * n_tiles_n;
        const int g = wgid / per_group, loc = wgid - g * per_group;
        const int gm = min(GM, n_tiles_m - g * GM);
        const int tn = loc / gm;
        m0 = (g * GM + (loc - tn * gm)) * BM;
        n0 = tn * BM;
    };
    // LDS-DMA: buffer_load_dwordx4 ... lds (32-bit lane offsets into a per-tile panel buffer
    // descriptor, k0 in the scalar offset).  Both operands are interleaved two-part images
    // (common.h, kx == 2): one K-step of a row is one 128-B line [hi 32 | lo 32], so a 1 KiB piece
    // is 8 rows x 128 B — whole-line requests (round 6: the planar images took 16 rows x 64 B
    // per piece, two half-line requests per row and K-step; the K loop is request-rate bound,
    // profiles/r5kline_fullline_dma.txt).  In LDS each operand is 256 rows at a 128-B pitch, chunk
    // c (0-3 hi, 4-7 lo) of row n at slot c ^ ((n >> 1) & 7).  Wave w stages pieces p = 0..7:
    // operand p >> 2 (A, W), rows n = 128 (p & 1) + 16 w + 8 ((p >> 1) & 1) + (lane >> 3), lane
    // slot lane & 7 (its logical chunk swizzled on the source address).
    const size_t ld2 = (size_t)2 * K;
    __amdgpu_buffer_rsrc_t rsA, rsW;
    int voffA[4], voffW[4];                       // lane byte offsets: (p & 1) row half x 8-row half
    // VAR 16777216: output columns permuted inside each 32-column group so that a lane's two
    // 16-column MFMA blocks 2m, 2m + 1 hold 8 CONSECUTIVE output columns (32 m + 8 q4 .. + 7)
    // instead of two runs of 4: W image row 32 m + 16 jj + 4 q + e is W row 32 m + 8 q + 4 jj + e.
    // The epilogue's per-lane loads (bias, residual image, LayerNorm weights) become 16-B loads.
    constexpr bool PERM = (VAR & 16777216) != 0;
    constexpr bool RESDMA = LNR && (VAR & 4) != 0;     // the LayerNorm epilogue's residual by LDS-DMA
    auto wperm = [](int L) {
        return PERM ? (L & ~31) | (((L >> 2) & 3) << 3) | (((L >> 4) & 1) << 2) | (L & 3) : L;
    };
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int l = 0; l < 2; ++l) {
            const int n = 128 * h + wave * 16 + 8 * l + (lane >> 3);
            const int sl = ((lane & 7) ^ ((n >> 1) & 7)) * 8;
            voffA[2 * h + l] = (n * (int)ld2 + sl) * 2;
            voffW[2 * h + l] = (wperm(n) * ldw + sl) * 2;
        }
    auto set_rsrc = [&](int m0, int n0) {
        rsA = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (size_t)m0 * ld2), (short)0, (int)(256 * ld2 * 2), 0x00020000);
        rsW = __builtin_amdgcn_make_buffer_rsrc((void*)(W + (size_t)n0 * ldw), (short)0, 256 * ldw * 2, 0x00020000);
    };
    auto piece = [&](int buf, int k0, int p) {
        if constexpr ((DV & 1) != 0) return;      // diagnostic: no K-loop staging (stale tiles)
        const int r = p >> 1;
        const int dofs = (r >> 1) * 2 * REG + ((p & 1) * 128 + wave * 16 + 8 * (r & 1)) * 128;
        auto* dst = (__attribute__((address_space(3))) void*)(smem + buf * STAGE + dofs);
        const int vo = (r < 2 ? voffA : voffW)[2 * (p & 1) + (r & 1)];
        // k0 halves of logical K = 2 k0 halves of the image = 4 k0 bytes.  The scalar offset is
        // outside the descriptor's range check (only the lane offset is checked): the host
        // guarantees K-step k0 lies inside every row (launch_gemm_x3s: ldw >= 2K)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r < 2 ? rsA : rsW, dst, 16, vo, k0 * 4, 0, 0);
    };
    auto stage = [&](int buf, int k0) {
#pragma unroll
        for (int p = 0; p < 8; ++p) piece(buf, k0, p);
    };
    const half8 up = (half8)(f16)X3_UP;

    // v_mfma_f32_16x16x32_f16, one MFMA per BK = 32 step.  Lane l supplies row (l & 15) of a
    // 16-row block at 16-B k-chunk (l >> 4): a wave reads the hi (or lo) halves of 16 rows per
    // ds_read_b128.  The chip holds a higher clock under the
    // 16x16 shape at equal MFMA cycles (MI355X_MICROARCH 'DVFS give-back' 7; +6-8 % over
    // 32x32x16 here).  acc16[i][j]: rows 16 i + (l & 15) of the wave tile, columns
    // 16 j + 4 (l >> 4) .. +3.  Per K-step: W_hi, W_lo of the wave's 64 columns once (+ 64 W_hi
    // in registers), then two halves of 4 row blocks each.
    // The three products at one scale, 64x the value: (64 W_hi) A_hi + W_hi (64 A_lo) + (64 W_lo) A_hi
    // (the images hold the lo parts x64), so the accumulators carry 64 C and the epilogue scales
    // by 1/64 with its bias add.  One operand scaled in registers per K-step (16 v_pk_mul_f16 per
    // wave) instead of W_hi/64 and A_hi/64 (48; no scaling at all: the round-5 probe put those 48
    // at 2.4-2.9 % of the GEMM, profiles/r5t_x3s_scale.txt) — and no operand is divided down
    // toward the fp16 subnormals the MFMA flushes.  64 W_hi must stay finite: |W_hi| <= 1023.5,
    // which rs_model_finalize checks before it packs a model's split-operand weights.
    const int r16 = lane & 15, q4 = lane >> 4;
    // fragment rows at a 128-B pitch: lane (r16, q4) reads hi chunk q4 of its row at slot
    // q4 ^ ((r16 >> 1) & 7); its lo chunk q4 + 4 is that slot ^ 4 (offset ^ 64).  The 16 lanes of a
    // ds_read_b128 group cover rows r16 = 0..15 at bank offsets 32 (r16 & 1) + 4 slot: conflict-free
    const int offA16 = (wm * WTM + r16) * 128 + ((q4 ^ ((r16 >> 1) & 7)) << 4);
    const int offW16 = 2 * REG + (wn * WTN + r16) * 128 + ((q4 ^ ((r16 >> 1) & 7)) << 4);
    f32x4 acc16[8][4];
    // the next step's eight DMA pieces ride this step's first MFMA groups (one per group of four
    // MFMAs of row half 0); the last step of a tile passes k0n = 2^29 and issues none (the same
    // pieces without their branches — against a zero-size descriptor on the last step — made
    // hipcc spill 10 / 19 VGPRs in the fp32 / GELU instances)
    auto kstep16 = [&](int buf, int k0n) {
        const char* sb = smem + buf * STAGE;
        half8 wh[4], wl[4], wu[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            wh[j] = *(const half8*)(sb + offW16 + j * 2048);
            wl[j] = *(const half8*)(sb + (offW16 ^ 64) + j * 2048);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) wu[j] = wh[j] * up;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            half8 ah[4], al[4];
#pragma unroll
            for (int ii = 0; ii < 4; ++ii) {
                ah[ii] = *(const half8*)(sb + offA16 + (4 * h + ii) * 2048);
                al[ii] = *(const half8*)(sb + (offA16 ^ 64) + (4 * h + ii) * 2048);
            }
#pragma unroll
            for (int pr = 0; pr < 3; ++pr) {
#pragma unroll
                for (int ii = 0; ii < 4; ++ii) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const half8 b = pr == 0 ? wu[j] : pr == 1 ? wh[j] : wl[j];
                        const half8 a = pr == 1 ? al[ii] : ah[ii];
                        acc16[4 * h + ii][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b, a, acc16[4 * h + ii][j], 0, 0, 0);
                    }
                    const int grp = 12 * h + 4 * pr + ii;
                    if (grp < 8 && k0n < (1 << 29)) {
                        __builtin_amdgcn_sched_barrier(0);
                        piece(buf ^ 1, k0n, grp);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
            }
        }
    };

    int m0, n0;
    tile_of(t, m0, n0);
    set_rsrc(m0, n0);
    stage(0, 0);
    int par = 0;                                                  // buffer of K-step 0
    bool first = true;
    for (;;) {
        // LNR, the last tile of the gang's panel list: column tile 0's wave 0 takes the next list
        // now (the youngest memory operation here: its return is waited for by K-step 1, a step
        // later) and hands it over at the transition
        unsigned nlist = 0;
        if constexpr (LNR) {
            if (m0 / BM + (int)gridDim.x / n_tiles_n >= n_tiles / n_tiles_n && n0 == 0 && wave == 0 && lane == 0)
                nlist = lnr_add(ep.lncnt, LNC_GANGS);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc16[i][j] = (f32x4)(0.f);
        // step kt landed for this wave (at a tile's first step the previous tile's stores are
        // younger and stay in flight); the barrier: landed for every wave, and every wave is done
        // reading step kt-1's buffer, which now receives step kt+1.  (DV 8, diagnostic: the DMA is
        // never waited for — isolates its latency from its presence.)
        int kt0 = 0;
        if constexpr (LNR) {
            // K-step 0 peeled with its next-step offset a constant (nk >= 2: launch_x3s): left to the
            // compiler, the peeled step tested a hoisted loop-invariant flag that this build spilled,
            // and the reload's vmcnt(0) drained the previous tile's 32 epilogue stores at every tile
            // start (the fp32 / GELU builds keep the loop: peeled by hand they spill)
            if constexpr ((DV & 8) == 0) {
                if (!first) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NSTORE) : "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            asm volatile("s_barrier" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            kstep16(par, BK);
            __builtin_amdgcn_sched_barrier(0);
            stamp(9);                                             // (stamp build) K-step 0
            kt0 = 1;
        }
        for (int kt = kt0; kt < nk; ++kt) {
            const int cur = (par + kt) & 1;
            if constexpr ((DV & 8) != 0) {
            } else if (kt == 0 && !first) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NSTORE) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("s_barrier" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            kstep16(cur, kt + 1 < nk ? (kt + 1) * BK : (1 << 29));
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (STAMP && !LNR) {
                if (kt == 0) stamp(9);                            // (stamp build) K-step 0
            }
        }
        stamp(0);                                                 // K loop
        // ---- transition
        const int last = (par + nk - 1) & 1;                      // buffer of the last K-step
        const int cm0 = m0, cn0 = n0;
        // bias of this tile (16-B quads of the lane's 4 consecutive columns, 16 j + 4 (l >> 4) of
        // the wave's 64): only the bias loads (and, LayerNorm build, the residual's first pieces)
        // are outstanding here (the last K-step issued no DMA), so one vmcnt(0) waits for exactly
        // them; inline asm keeps the compiler from placing its own wait
        // LayerNorm build (VAR 4): the residual's first two row blocks go out as LDS-DMA before the
        // bias loads, so their latency and the bias loads' overlap (lnres_epilogue streams the rest)
        const int rbo = (last ^ 1) * STAGE + wave * 8192;
        const __amdgpu_buffer_rsrc_t rsR = __builtin_amdgcn_make_buffer_rsrc(
            (void*)((const f16*)ep.out + (size_t)cm0 * ep.ldc), (short)0, 256 * ep.ldc * 2, 0x00020000);
        int voR[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {            // q = 2 m + hf: 32-column group m, row half hf
            const int jr = 8 * (q & 1) + (lane >> 3);
            const int cc = (lane & 7) ^ ((jr >> 1) & 7);
            voR[q] = ((wm * WTM + jr) * ep.ldc + 2 * (cn0 + wn * WTN) + 64 * (q >> 1) + 8 * cc) * 2;
        }
        auto issue = [&](int rb) __attribute__((always_inline)) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                auto* dst = (__attribute__((address_space(3))) void*)(smem + rbo + (rb & 1) * 4096 + q * 1024);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsR, dst, 16, voR[q], rb * 16 * ep.ldc * 2, 0, 0);
            }
        };
        if constexpr (RESDMA) {
            issue(0);
            issue(1);
        }
        f32x4 bq[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float* bp = ep.bias + cn0 + wn * WTN + (PERM ? 32 * (j >> 1) + 8 * q4 + 4 * (j & 1) : 16 * j + 4 * q4);
            asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(bq[j]) : "v"(bp) : "memory");
        }
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(bq[0]), "+v"(bq[1]), "+v"(bq[2]), "+v"(bq[3]) : : "memory");
        // the next tile's stage 0 (into the buffer step nk-2 used) lands while this epilogue runs
        // (issuing it after the LayerNorm epilogue's residual loads instead, so that their waits
        // need not cover this DMA, measured -2.7 %: profiles/r3p2_lnperm_ab.txt)
        bool more = false;
        t += gridDim.x;
        if constexpr (LNR) {
            if (t >= n_tiles && !lnr_next_list(ep, t, nlist, cm0 / BM, cn0 / BM, n_tiles_n, n_tiles, wave, lane)) break;
        }
        more = t < n_tiles;
        // VAR 1073741824 (the LayerNorm build's default): the next tile's stage 0 issued after the
        // row statistics instead (lnres_epilogue's caller) — its eight back-to-back DMA issues cost
        // this phase ~6k cycles per tile here, where nothing hides them (the residual phase is
        // unchanged either way; profiles/r5late0_stage0_after_stats.txt).  It still lands before the
        // next tile's K-step 0, whose vmcnt(NSTORE) leaves only the younger epilogue stores in flight.
        constexpr bool LATE0 = LNR && (VAR & 1073741824) != 0;
        if (more) {
            tile_of(t, m0, n0);
            set_rsrc(m0, n0);
            if constexpr (!LATE0) stage(last ^ 1, 0);
        }
        stamp(1);                                                 // bias wait + next tile's stage 0
        // bias (+ GELU) of row blocks [i0, i1)
        auto finish = [&](int i0, int i1) {
#pragma unroll
            for (int i = i0; i < i1; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int e = 0; e < 4; e += 2) {
                        // the accumulators hold 64 C (kstep16): C + bias in one packed FMA
                        f32x2 v = __builtin_elementwise_fma((f32x2){acc16[i][j][e], acc16[i][j][e + 1]}, (f32x2)(X3_DOWN),
                                                            (f32x2){bq[j][e], bq[j][e + 1]});
                        if constexpr (EPI == EPI_GELU_F16) v = gelu2(v);
                        acc16[i][j][e] = v.x;
                        acc16[i][j][e + 1] = v.y;
                    }
        };
            auto lnres_epilogue = [&]() {
                const int H = ep.nlog, ldc = ep.ldc, ntn = n_tiles_n;
                const int panel = cm0 / BM, tcol = cn0 / BM;
                const unsigned long long tag = (unsigned long long)ep.ln_tag << 32;
                const f16* img = (const f16*)ep.out;
                const int c0 = cn0 + wn * WTN + 4 * q4;
                // x = (acc + bias) + h, the residual image h = hi + lo/64 read in the accumulator
                // layout, four row blocks at a time (as ln_res_img forms it); the permuted-column
                // layout (PERM) halves its load count: +1.1 % end to end.  (Reading it during the K
                // loop instead, one row block per K-step added into the accumulators, measured
                // neutral — 63,277 vs 63,263 masked fwd/s, profiles/r5b_lnkres_ab.txt — and made a
                // row's sum depend on its position in the tile, so it was removed.)
                // (two row blocks per batch: four would hold 64 registers of residual beside the 128
                // accumulators, and the spills that forced reloaded values whose waits drained the
                // next tile's stage 0 inside the statistics publish)
                constexpr int RB2 = 2;
                // per row block: acc <- acc / 64 + bias + (hi + lo/64) from packed (hi, lo) fp16 pairs
                auto add_res = [&](int rb, const half4 (&rh)[4], const half4 (&rl)[4]) __attribute__((always_inline)) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        // h = hi + lo/64 by v_fma_mix on the packed fp16 parts (gemm_dev.h mix_val)
                        const uint2 hv = __builtin_bit_cast(uint2, rh[j]), lv = __builtin_bit_cast(uint2, rl[j]);
                        const float hres[4] = {mix_val<0>(hv.x, lv.x, X3_DOWN), mix_val<1>(hv.x, lv.x, X3_DOWN),
                                               mix_val<0>(hv.y, lv.y, X3_DOWN), mix_val<1>(hv.y, lv.y, X3_DOWN)};
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            acc16[rb][j][e] = __builtin_fmaf(acc16[rb][j][e], X3_DOWN, bq[j][e]) + hres[e];
                    }
                };
                if constexpr (RESDMA) {
                    // VAR 4: the residual by whole-line LDS-DMA pieces (8 rows x 128 B, as the K loop
                    // stages its operands) into this wave's 8 KiB of the NEXT tile's stage-0 buffer —
                    // free here: its last reads (K-step nk - 2) are behind the last K-step's barrier, and
                    // LATE0 issues stage 0 into it only after the statistics.  Two row blocks in
                    // flight; the lane reads its (hi, lo) 16-B chunks back in the accumulator layout
                    // (chunk c of LDS row n at c ^ ((n >> 1) & 7), as the K loop's images).
                    // (pieces of row blocks 0 and 1 issued at the transition, before the bias loads)
                    static_assert(!RESDMA || (LATE0 && PERM), "the residual DMA needs the late stage 0");
                    const uint32_t lrow = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem + rbo +
                                          r16 * 128;
                    const uint32_t lh = lrow + ((q4 ^ ((r16 >> 1) & 7)) << 4), ll = lrow + (((q4 + 4) ^ ((r16 >> 1) & 7)) << 4);
#pragma unroll
                    for (int rb = 0; rb < 8; ++rb) {
                        if (rb < 7) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        uint4 h0, h1, l0, l1;                 // (hi, lo) of groups m = 0, 1
                        const int so = (rb & 1) * 4096;
                        asm volatile(
                            "ds_read_b128 %0, %4 offset:%6\n\t"
                            "ds_read_b128 %1, %4 offset:%7\n\t"
                            "ds_read_b128 %2, %5 offset:%6\n\t"
                            "ds_read_b128 %3, %5 offset:%7\n\t"
                            "s_waitcnt lgkmcnt(0)"
                            : "=&v"(h0), "=&v"(h1), "=&v"(l0), "=&v"(l1)
                            : "v"(lh), "v"(ll), "i"(so), "i"(so + 2048)
                            : "memory");
                        if (rb + 2 < 8) issue(rb + 2);
                        const half8 vh0 = __builtin_bit_cast(half8, h0), vh1 = __builtin_bit_cast(half8, h1);
                        const half8 vl0 = __builtin_bit_cast(half8, l0), vl1 = __builtin_bit_cast(half8, l1);
                        const half4 rh[4] = {(half4){vh0[0], vh0[1], vh0[2], vh0[3]}, (half4){vh0[4], vh0[5], vh0[6], vh0[7]},
                                             (half4){vh1[0], vh1[1], vh1[2], vh1[3]}, (half4){vh1[4], vh1[5], vh1[6], vh1[7]}};
                        const half4 rl[4] = {(half4){vl0[0], vl0[1], vl0[2], vl0[3]}, (half4){vl0[4], vl0[5], vl0[6], vl0[7]},
                                             (half4){vl1[0], vl1[1], vl1[2], vl1[3]}, (half4){vl1[4], vl1[5], vl1[6], vl1[7]}};
                        add_res(rb, rh, rl);
                    }
                }
#pragma unroll
                for (int hh = 0; hh < (RESDMA ? 0 : 8 / RB2); ++hh) {
                    half4 rh0[RB2][4], rl0[RB2][4];
#pragma unroll
                    for (int ii = 0; ii < RB2; ++ii) {
                        // the interleaved image row: column c's hi at il_hi(c), its lo 32 halves on
                        const f16* prow_img = img + (size_t)(cm0 + wm * WTM + 16 * (RB2 * hh + ii) + r16) * ldc;
                        if constexpr (PERM) {
                            // blocks 2m, 2m + 1: 8 consecutive columns (32-column group m of the
                            // wave's 64), one 16-B load per part
#pragma unroll
                            for (int m = 0; m < 2; ++m) {
                                const f16* p = prow_img + 2 * (cn0 + wn * WTN) + 64 * m + 8 * q4;
                                const half8 vh = *(const half8*)p, vl = *(const half8*)(p + 32);
                                rh0[ii][2 * m] = (half4){vh[0], vh[1], vh[2], vh[3]};
                                rh0[ii][2 * m + 1] = (half4){vh[4], vh[5], vh[6], vh[7]};
                                rl0[ii][2 * m] = (half4){vl[0], vl[1], vl[2], vl[3]};
                                rl0[ii][2 * m + 1] = (half4){vl[4], vl[5], vl[6], vl[7]};
                            }
                        } else {
#pragma unroll
                            for (int j = 0; j < 4; ++j) {
                                const f16* p = prow_img + il_hi(c0 + 16 * j);
                                rh0[ii][j] = *(const half4*)p;
                                rl0[ii][j] = *(const half4*)(p + 32);
                            }
                        }
                    }
#pragma unroll
                    for (int ii = 0; ii < RB2; ++ii) add_res(RB2 * hh + ii, rh0[ii], rl0[ii]);
                }
                stamp(2);                                         // residual read + add
                // row partials over the wave's 64 columns (lanes l, l^16, l^32, l^48 share a row),
                // then over the four waves of the row half through their slabs
                float* red = (float*)(slabs + wave * 4096);
                auto slab_of = [&](int w2) { return (const float*)(slabs + (wm * WN + w2) * 4096); };
                float tmean[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    float a = 0.f;
#pragma unroll
                    for (int j = 0; j < 4; ++j) a += (acc16[i][j][0] + acc16[i][j][1]) + (acc16[i][j][2] + acc16[i][j][3]);
                    a += __shfl_xor(a, 16);
                    a += __shfl_xor(a, 32);
                    tmean[i] = a;
                }
                if (q4 == 0) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) red[16 * i + r16] = tmean[i];
                }
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    float a = 0.f;
#pragma unroll
                    for (int w2 = 0; w2 < WN; ++w2) a += slab_of(w2)[16 * i + r16];
                    tmean[i] = a * (1.f / BM);
                }
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    float q = 0.f;
#pragma unroll
                    for (int j = 0; j < 4; ++j)
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const float d = acc16[i][j][e] - tmean[i];
                            q = __builtin_fmaf(d, d, q);
                        }
                    q += __shfl_xor(q, 16);
                    q += __shfl_xor(q, 32);
                    if (q4 == 0) red[128 + 16 * i + r16] = q;
                }
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
                // waves wn == 0: lane l owns rows l and l + 64 of the row half — its tile partials
                // from the slabs (the same sums in the same order for every wave), published as
                // granules, the peers' polled, the row statistics combined into the ring buffer
                // this tile's last K-step read (free until the next tile's first barrier; the
                // slabs are rewritten by the store pass)
                float2* st2 = (float2*)(smem + last * STAGE) + wm * WTM;
                volatile unsigned* bailw = (volatile unsigned*)(smem + last * STAGE + 4096);   // per row half
                if (wn == 0) {
                    typedef unsigned long long u64;
                    u64* gx = (u64*)ep.lnx + (size_t)panel * ntn * BM * 2 + wm * WTM * 2;   // [c][row][2]
                    // the lane's granule offsets formed here, per tile (opaque lane index): hoisted out
                    // of the tile loop they were a spilled 64-bit register whose reload waited for
                    // the next tile's stage 0 before every publish
                    int ln = lane;
                    asm volatile("" : "+v"(ln));
                    float os[2], oq[2];
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const int rr = ln + 64 * k;
                        float a = 0.f, b = 0.f;
#pragma unroll
                        for (int w2 = 0; w2 < WN; ++w2) {
                            a += slab_of(w2)[rr];
                            b += slab_of(w2)[128 + rr];
                        }
                        os[k] = a;
                        oq[k] = b;
                        u64* g = gx + ((size_t)tcol * BM + rr) * 2;
                        __hip_atomic_store((gu64*)g, tag | __float_as_uint(a), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store((gu64*)(g + 1), tag | __float_as_uint(b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    float ps[2][4], pq[2][4];
                    bool failed = false;
                    stamp(3);                                     // tile statistics + publish (wave 0)
                    const unsigned long long t_lim = lnr_wait_ticks(ep.diag), t_start = lnr_now();
                    for (unsigned spins = 0;;) {
                        bool ok = true;
#pragma unroll
                        for (int k = 0; k < 2; ++k)
#pragma unroll
                            for (int c = 0; c < 4; ++c) {
                                ps[k][c] = os[k];
                                pq[k][c] = oq[k];
                                if (c < ntn && c != tcol) {
                                    const u64* g = gx + ((size_t)c * BM + ln + 64 * k) * 2;
                                    const u64 va = __hip_atomic_load((const gu64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                    const u64 vb = __hip_atomic_load((const gu64*)(g + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                    ok &= (va >> 32) == (tag >> 32) && (vb >> 32) == (tag >> 32);
                                    ps[k][c] = __uint_as_float((unsigned)va);
                                    pq[k][c] = __uint_as_float((unsigned)vb);
                                }
                            }
                        if (ep.diag & 8) ok = false;        // diag 8 (tests): peers never arrive
                        if (__all(ok)) break;
                        __builtin_amdgcn_s_sleep(1);
                        // bounded: a wait that cannot end (the gang's workgroups not co-resident)
                        // sets the sticky error word; a wait that sees the word set (another
                        // workgroup timed out) gives up too, so the launch drains fast
                        if ((++spins & 63) == 0 &&
                            (lnr_now() - t_start > t_lim ||
                             __hip_atomic_load((const gu32*)ep.lnerr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
                            if (lane == 0) __hip_atomic_store((gu32*)ep.lnerr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            failed = true;
                            break;
                        }
                    }
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const float inv_n = 1.f / H;
                        float tot = 0.f;
#pragma unroll
                        for (int c = 0; c < 4; ++c)
                            if (c < ntn) tot += ps[k][c];
                        const float mean = tot * inv_n;
                        float m2 = 0.f;
#pragma unroll
                        for (int c = 0; c < 4; ++c) {
                            if (c < ntn) {
                                const float d = ps[k][c] * (1.f / BM) - mean;
                                m2 += __builtin_fmaf((float)BM * d, d, pq[k][c]);
                            }
                        }
                        st2[lane + 64 * k] = make_float2(mean, 1.0f / sqrtf(__builtin_fmaf(m2, inv_n, ep.ln_eps)));
                    }
                    if (lane == 0) bailw[wm] = failed ? 1u : 0u;
                    stamp(4);                                     // peers' statistics (poll)
                }
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
                if (bailw[0] | bailw[1]) return true;    // a wait gave up: the launch drains (RS_EHIP)
                f32x4 gq[4], bb[4];                      // LayerNorm weight / bias of the lane's columns
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int cj = PERM ? cn0 + wn * WTN + 32 * (j >> 1) + 8 * q4 + 4 * (j & 1) : c0 + 16 * j;
                    gq[j] = *(const f32x4*)(ep.res_g + cj);
                    bb[j] = *(const f32x4*)(ep.res_b + cj);
                }
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const float2 st = st2[16 * i + r16];
#pragma unroll
                    for (int j = 0; j < 4; ++j)
#pragma unroll
                        for (int e = 0; e < 4; ++e) acc16[i][j][e] = ln_apply(acc16[i][j][e], st, gq[j][e], bb[j][e]);
                }
                stamp(5);                                         // barrier, LN weights, LN apply
                return false;
            };
            // the GELU image: each row-block pair's bias + GELU right before its slab pass, so that
            // VALU work overlaps the previous pair's LDS and global stores
            constexpr bool LATE = EPI == EPI_GELU_F16 && (DV & 2) == 0;
            if constexpr (LNR) {
                if (lnres_epilogue()) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the next tile's stage 0 landed
                    break;
                }
                if constexpr (LATE0) {
                    if (more) stage(last ^ 1, 0);
                }
            } else if constexpr (!LATE) finish(0, 8);
            if constexpr ((DV & 2) != 0) {       // diagnostic: no epilogue stores (acc kept alive)
#pragma unroll
                for (int i = 0; i < 8; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc16[i][j]));
                if (!more) break;
                par = last ^ 1;
                first = false;
                continue;
            }
            char* slb = slabs + wave * 4096;
            // (LayerNorm build: the store pass's lane offsets formed per tile — hoisted, they were a
            // spilled register reloaded inside the residual wait)
            int lns = lane;
            if constexpr (LNR) asm volatile("" : "+v"(lns));
            const int rr0 = lns >> 3, c16 = lns & 7;
            // DV 33554432 (diagnostic): every tile stores onto the rows of row panel 0
            const int sm0 = (DV & 33554432) ? 0 : cm0;
            if constexpr (EPI == EPI_BIAS_F32) {
                // 32 x 32 fp32 slab blocks: row blocks 2 i2 + a, column blocks 2 j2 + b
#pragma unroll
                for (int i2 = 0; i2 < 4; ++i2)
#pragma unroll
                    for (int j2 = 0; j2 < 2; ++j2) {
#pragma unroll
                        for (int a = 0; a < 2; ++a)
#pragma unroll
                            for (int b = 0; b < 2; ++b) {
                                const int row = 16 * a + r16, ch = 4 * b + q4;
                                *(f32x4*)(slb + row * 128 + ((ch ^ (row & 7)) << 4)) = acc16[2 * i2 + a][2 * j2 + b];
                            }
                        float* ob = (float*)ep.out + (size_t)(sm0 + wm * WTM + 32 * i2) * ep.ldc + cn0 + wn * WTN + 32 * j2 + 4 * c16;
                        uint4 v[4];
                        slab_read4(slb, rr0, c16, v);
#pragma unroll
                        for (int it = 0; it < 4; ++it) st16<64>((uint4*)(ob + (size_t)(it * 8 + rr0) * ep.ldc), v[it]);
                    }
            } else {
                // the interleaved two-part image in 32 x 64 slab blocks: row blocks 2 i2 + a, one
                // 32-column group g of the wave's 64 per block, each slab row its 128-B line
                // [hi 32 | lo*64 32] (column blocks 2 g, 2 g + 1)
                // row-block pair outermost: its accumulators die after both groups are out
#pragma unroll
                for (int i2 = 0; i2 < 4; ++i2) {
                    if constexpr (LATE) finish(2 * i2, 2 * i2 + 2);
#pragma unroll
                    for (int g = 0; g < 2; ++g) {
#pragma unroll
                        for (int a = 0; a < 2; ++a)
#pragma unroll
                            for (int jj = 0; jj < 2; ++jj) {
                                // hi = RNE(x) (v_cvt_pk_f16_f32), lo = RNE(64 x - 64 hi) (mix_lo2)
                                half4 hh, hl;
                                const f32x4 xv = acc16[2 * i2 + a][2 * g + jj];
#pragma unroll
                                for (int e = 0; e < 4; ++e) hh[e] = (f16)xv[e];
                                const uint2 hv = __builtin_bit_cast(uint2, hh);
                                const f32x2 s01 = (f32x2){xv[0], xv[1]} * X3_UP, s23 = (f32x2){xv[2], xv[3]} * X3_UP;
                                hl = __builtin_bit_cast(half4, (uint2){mix_lo2(hv.x, s01.x, s01.y, -X3_UP),
                                                                       mix_lo2(hv.y, s23.x, s23.y, -X3_UP)});
                                const int row = 16 * a + r16, byte = PERM ? 16 * q4 + 8 * jj : 32 * jj + 8 * q4;
                                *(half4*)(slb + row * 128 + (((byte >> 4) ^ (row & 7)) << 4) + (byte & 8)) = hh;
                                *(half4*)(slb + row * 128 + ((((byte >> 4) + 4) ^ (row & 7)) << 4) + (byte & 8)) = hl;
                            }
                        f16* ob = (f16*)ep.out + (size_t)(sm0 + wm * WTM + 32 * i2) * ep.ldc + 2 * (cn0 + wn * WTN) + 64 * g + 8 * c16;
                        uint4 v[4];
                        slab_read4(slb, rr0, c16, v);
#pragma unroll
                        for (int it = 0; it < 4; ++it) st16<64>((uint4*)(ob + (size_t)(it * 8 + rr0) * ep.ldc), v[it]);
                    }
                }
            }
            stamp(6);                                             // epilogue stores
            if constexpr (STAMP) st_sum[7] += 1;
            if (!more) break;
            par = last ^ 1;
            first = false;
    }
    if constexpr (STAMP) {
        if (tid == 0) {
#pragma unroll
            for (int ph = 0; ph < 10; ++ph) ep.dbg[blockIdx.x * 16 + ph] += st_sum[ph];
        }
    }
    if constexpr (LNR) {
        if (tid == 0) lnr_done(ep);
    }
}

// Sequence number of a LayerNorm-epilogue launch (the granule tag), process-wide: never 0.
unsigned ln_tag_next() {
    static std::atomic<unsigned> seq{0};
    unsigned v = seq.fetch_add(1, std::memory_order_relaxed) + 1;
    while (v == 0) v = seq.fetch_add(1, std::memory_order_relaxed) + 1;
    return v;
}

int n_cus() {
    static int n = [] {
        int dev = 0, v = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
        return v > 0 ? v : 256;
    }();
    return n;
}

// Raise a kernel's dynamic-LDS limit once per device (the attribute is per device; a process may
// drive several).
hipError_t smem_attr_once(const void* fn, int smem, std::atomic<unsigned>& devs) {
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev)) return e;
    const unsigned bit = 1u << (dev & 31);
    if (devs.load(std::memory_order_acquire) & bit) return hipSuccess;
    if (hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, smem)) return e;
    devs.fetch_or(bit, std::memory_order_release);
    return hipSuccess;
}

template <int EPI, int VAR = 0>
hipError_t launch_x3s(const f16* A, const f16* W, int M_pad, int N_pad, int K, const EpiArgs& ep, hipStream_t st,
                      int ldw = 0) {
    constexpr int smem = 2 * 65536;                  // ring (2 x 64 KiB); + 32 KiB static wave slabs
    if (K % 32 || K < 64 || M_pad % 256 || N_pad % 256) return hipErrorInvalidValue;
    static std::atomic<unsigned> attr_devs{0};      // devices whose LDS limit is raised
    if (hipError_t e = smem_attr_once((const void*)gemm_x3s_kernel<EPI, VAR>, smem, attr_devs)) return e;
    const int ntn = N_pad / 256, n_tiles = (M_pad / 256) * ntn;
    const int cus = n_cus() / 8 * 8;
    int grid = n_tiles <= cus ? n_tiles : cus;
    if constexpr (EPI == EPI_LNRES_IMG) {
        // the image is rewritten in place over whole rows (N_pad = the hidden size, <= 4 column
        // tiles); the ticket words are zero at every launch (lnr_done)
        if (!ep.lnx || !ep.lncnt || !ep.lnerr || N_pad > 1024 || ep.nlog != N_pad || ep.ldc != 2 * N_pad)
            return hipErrorInvalidValue;
        // whole row panels per round: the first tiles form complete gangs (every workgroup
        // resident at one per CU)
        grid = std::min(n_tiles, cus / ntn * ntn);
    }
    static const int gm_env = getenv("RS_GEMM_GROUP_M_X3S") ? atoi(getenv("RS_GEMM_GROUP_M_X3S")) : 0;
    EpiArgs e2 = ep;
    e2.group_m = gm_env > 0 ? gm_env : 8;
    if constexpr (EPI == EPI_LNRES_IMG) {
        // granule tag: this launch's sequence number (never 0: the granules start zeroed), so a
        // granule left by an earlier launch never matches.  One counter for every instance of the
        // kernel (ln_tag_next): the O-projection and BertOutput instances share the granule buffer,
        // and per-instance counters would repeat each other's tags
        e2.ln_tag = ln_tag_next();
    }
    const int ldw2 = ldw > 0 ? ldw : 2 * K;
    hipLaunchKernelGGL((gemm_x3s_kernel<EPI, VAR>), dim3(grid), dim3(512), smem, st, A, W, K, ldw2, ntn, n_tiles, e2);
    return hipGetLastError();
}

template <int EPI, int VAR = 0>
hipError_t launch_persist(const f16* A, const f16* W, int M_pad, int N_pad, int K, const EpiArgs& ep,
                          hipStream_t st) {
    // VAR 1048576: wave-private epilogue slabs in their own 32 KiB after the ring (160 KiB)
    constexpr int smem = 2 * 512 * 64 * 2 + ((VAR & 1048576) ? 8 * 32 * 128 : 0);
    if (K % 64 || M_pad % 256 || N_pad % 256) return hipErrorInvalidValue;
    static std::atomic<unsigned> attr_devs{0};      // devices whose LDS limit is raised
    if (hipError_t e = smem_attr_once((const void*)gemm_persist_kernel<EPI, VAR>, smem, attr_devs)) return e;
    const int ntn = N_pad / 256, n_tiles = (M_pad / 256) * ntn;
    const int cus = n_cus() / 8 * 8;
    const int grid = n_tiles <= cus ? n_tiles : cus;
    // 8 row panels per group (QKV -3 % vs 4, end to end; profiles/r1_ab_session2.txt)
    static const int gm_env = getenv("RS_GEMM_GROUP_M_P") ? atoi(getenv("RS_GEMM_GROUP_M_P")) : 0;
    // BertOutput (VAR tag 131072, K = 3072): RS_GEMM_GROUP_M_FFN2 row panels per group
    static const int gm_ffn2 = getenv("RS_GEMM_GROUP_M_FFN2") ? atoi(getenv("RS_GEMM_GROUP_M_FFN2")) : 0;
    EpiArgs e2 = ep;
    e2.group_m = (VAR & 131072) && gm_ffn2 > 0 ? gm_ffn2 : gm_env > 0 ? gm_env : 8;
    hipLaunchKernelGGL((gemm_persist_kernel<EPI, VAR>), dim3(grid), dim3(512), smem, st, A, W, K, ntn, n_tiles, e2);
    return hipGetLastError();
}

// name tags (kernel names only): 1 = O projection (VAR 65536), 2 = BertOutput (VAR 131072)
template <int EPI, int V>
hipError_t persist_tagged(int tag, const f16* A, const f16* W, int M_pad, int N_pad, int K, const EpiArgs& ep,
                          hipStream_t st) {
    return tag == 1 ? launch_persist<EPI, V | 65536>(A, W, M_pad, N_pad, K, ep, st)
         : tag == 2 ? launch_persist<EPI, V | 131072>(A, W, M_pad, N_pad, K, ep, st)
                    : launch_persist<EPI, V>(A, W, M_pad, N_pad, K, ep, st);
}

template <int BM, int BN, int WM, int WN, int NSTAGE, int BK, int EPI, int VAR = 0>
hipError_t launch_t(const f16* A, const f16* W, int M_pad, int N_pad, int K, const EpiArgs& ep,
                    hipStream_t st) {
    constexpr int smem = NSTAGE * (BM + BN) * BK * 2;
    if (K % BK) return hipErrorInvalidValue;
    static std::atomic<unsigned> attr_devs{0};      // devices whose LDS limit is raised
    if (hipError_t e = smem_attr_once((const void*)gemm_f16_kernel<BM, BN, WM, WN, NSTAGE, BK, EPI, VAR>, smem, attr_devs)) return e;
    const int ntn = N_pad / BN;
    const int grid = (M_pad / BM) * ntn;
    static const int gm_env = getenv("RS_GEMM_GROUP_M") ? atoi(getenv("RS_GEMM_GROUP_M")) : 0;
    EpiArgs e2 = ep;
    e2.group_m = gm_env > 0 ? gm_env : 4;   // 4 row panels per group (measured best of 1/2/4/8/16)
    hipLaunchKernelGGL((gemm_f16_kernel<BM, BN, WM, WN, NSTAGE, BK, EPI, VAR>), dim3(grid), dim3(WM * WN * 64),
                       smem, st, A, W, K, ntn, e2);
    return hipGetLastError();
}

// fp16-operand GEMMs (the fp16 precision mode, the K-concatenated fp16x3 form RS_X3S=0, the
// last layer's query rows and the MLM head), the measured-best variant per epilogue:
//   * bias / GELU fp16 outputs (kx = 1): the persistent kernel, younger wave half at s_setprio 1
//     and one MFMA substep behind, wave-private epilogue slabs without the epilogue barrier for
//     the bias epilogue (VAR 786432 | 1048576; +1.2 / +1.5 / +1.6-1.9 %, profiles/r1_session3_probes.txt);
//   * the GELU three-part image of the K-concatenated fp16x3 form: the persistent kernel (VAR 4194304);
//   * everything else (fp32 outputs, the residual epilogues, the decoder logsumexp): the pipelined
//     256 x 256 (N % 256 == 0) or 256 x 128 kernel, 16x16x32 MFMA except the logsumexp epilogue
//     (32x32x16), non-temporal stores for fp16 outputs (VAR 64).
// Measured-slower alternatives (tile configurations 2-7, 32x32x16 in the pipelined kernel, the
// unstaggered persistent schedules, direct residual stores, ...) are recorded in profiles/r1_*;
// their code paths were removed in round 4.
template <int EPI>
hipError_t launch_epi(const f16* A, const f16* W, int M_pad, int N_pad, int K, const EpiArgs& ep,
                      hipStream_t st, int tag) {
    const bool n256 = N_pad % 256 == 0;
    if constexpr (EPI == EPI_GELU_F16) {
        if (n256 && ep.kx == 3) return launch_persist<EPI, 786432 | 4194304>(A, W, M_pad, N_pad, K, ep, st);
    }
    if constexpr (EPI == EPI_BIAS_F16 || EPI == EPI_GELU_F16) {
        if (n256 && (EPI == EPI_BIAS_F16 || ep.kx == 1)) {
            constexpr int SLAB = EPI == EPI_BIAS_F16 ? 1048576 : 0;
            return persist_tagged<EPI, 786432 | SLAB>(tag, A, W, M_pad, N_pad, K, ep, st);
        }
        if (n256) return launch_t<256, 256, 2, 4, 2, 64, EPI, 192 | 8192>(A, W, M_pad, N_pad, K, ep, st);
        return launch_t<256, 128, 4, 2, 3, 64, EPI, 192 | 8192>(A, W, M_pad, N_pad, K, ep, st);
    } else if constexpr (EPI == EPI_LSE) {
        if (n256) return launch_t<256, 256, 2, 4, 2, 64, EPI, 128>(A, W, M_pad, N_pad, K, ep, st);
        return launch_t<256, 128, 4, 2, 3, 64, EPI, 128>(A, W, M_pad, N_pad, K, ep, st);
    } else {
        if (n256) return launch_t<256, 256, 2, 4, 2, 64, EPI, 128 | 8192>(A, W, M_pad, N_pad, K, ep, st);
        return launch_t<256, 128, 4, 2, 3, 64, EPI, 128 | 8192>(A, W, M_pad, N_pad, K, ep, st);
    }
}

}  // namespace

int gemm_row_align() { return 256; }

size_t lnres_counter_bytes() { return lnr_counter_bytes(); }

// Workgroups of one fused residual + LayerNorm GEMM launch (EPI_LNRES_IMG): whole gangs of the
// N_pad / 256 column tiles of a row panel, at one workgroup per CU.  A launch over P row panels
// runs ceil(P / gangs) rounds of panels, so the host cuts its chunks at multiples of
// 256 * gangs rows (run_all).
int gemm_lnres_workgroups(int N_pad) {
    const int ntn = N_pad / 256, cus = n_cus() / 8 * 8;
    return ntn > 0 ? cus / ntn * ntn : 0;
}

// Production split-operand fp16x3 GEMM (gemm_x3s_kernel; tools/x3s_epi_probe.py).
// Stamp builds (RS_DIAG only, rs_debug_stamps): while g_stamps is set, every split-operand GEMM
// launch runs the VAR 268435456 build of its kernel and adds its per-workgroup phase cycles into
// the region of its instance: 0 QKV / fp32 out, 1 BertIntermediate (GELU image), 2 O-projection +
// LayerNorm, 3 BertOutput + LayerNorm (each [256 workgroups][16 words]).
#if RS_DIAG
static unsigned long long* g_stamps = nullptr;
constexpr int STAMP_WORDS = 4 * 256 * 16;
#endif

template <int STV>
hipError_t launch_gemm_x3s_v(int epi, const f16* A, const f16* W, int ldw, int M_pad, int N_pad, int K,
                             const EpiArgs& ep_in, hipStream_t st) {
    EpiArgs ep = ep_in;
#if RS_DIAG
    if (STV) ep.dbg = g_stamps + (epi == EPI_BIAS_F32 ? 0 : epi == EPI_GELU_F16 ? 1 : K > 1024 ? 3 : 2) * 256 * 16;
#endif
    switch (epi) {
        case EPI_BIAS_F32: return launch_x3s<EPI_BIAS_F32, STV>(A, W, M_pad, N_pad, K, ep, st, ldw);
        case EPI_GELU_F16: return launch_x3s<EPI_GELU_F16, STV>(A, W, M_pad, N_pad, K, ep, st, ldw);
        case EPI_LNRES_IMG: {
            // Output columns permuted inside 32-column groups (VAR 16777216: 16-B epilogue loads,
            // +1.1 % end to end, profiles/r3p2_lnperm_ab.txt); VAR 67108864 is a name tag only (the
            // BertOutput launch, K = 3072), so rocprofv3 reports the two instances separately.
            // Gang formation (RS_LNGANG, read per call; lnr_gang_ticket): "xcd" (default) = start-order
            // tickets inside each XCD (VAR 134217728; a panel's column tiles share one L2), the rest
            // from an overflow ticket; "ticket" = consecutive start-order tickets.  Either way a
            // gang's members have all started before it exchanges statistics.  The exchange needs
            // ntn (= N_pad / 256) workgroups of the gang co-resident — anywhere on the GPU for
            // "ticket", on one XCD for "xcd" (or once the grid has started, anywhere): with fewer
            // free slots the bounded wait ends the call in RS_EHIP instead of hanging.
            // Default "xcd" (round 5: BertOutput fetch 25.0 -> 19.5 KB per row, O-projection 8.7 -> 7.2,
            // throughput within noise, profiles/r5d_gangs_pmc.txt); "ticket" needs the gang's
            // workgroups co-resident anywhere instead of on one XCD.
            const char* g = getenv("RS_LNGANG");
            const bool xcd = !(g && !strcmp(g, "ticket"));
            // VAR 1073741824: the next tile's stage 0 issued after the row statistics (O-projection
            // -1.1 %, BertOutput -0.7 %, profiles/r5late0_stage0_after_stats.txt)
            // VAR 4: the residual by whole-line LDS-DMA (round 6: O-projection -1.9 %, BertOutput -1.0 %,
            // C3 +0.4 %, bitwise; profiles/r6o_lnres_residual_dma.txt)
            constexpr int VL = 16777216 | 1073741824 | 4 | STV;
            if (xcd) {
                if (K > 1024) return launch_x3s<EPI_LNRES_IMG, VL | 67108864 | 134217728>(A, W, M_pad, N_pad, K, ep, st, ldw);
                return launch_x3s<EPI_LNRES_IMG, VL | 134217728>(A, W, M_pad, N_pad, K, ep, st, ldw);
            }
            if (K > 1024) return launch_x3s<EPI_LNRES_IMG, VL | 67108864>(A, W, M_pad, N_pad, K, ep, st, ldw);
            return launch_x3s<EPI_LNRES_IMG, VL>(A, W, M_pad, N_pad, K, ep, st, ldw);
        }
    }
    return hipErrorInvalidValue;
}

hipError_t launch_gemm_x3s(int epi, const f16* A, const f16* W, int ldw, int M_pad, int N_pad, int K,
                           const EpiArgs& ep, hipStream_t st) {
    if (M_pad % 256 || N_pad % 256 || K % 32 || K < 64 || ldw < 2 * K || M_pad <= 0) return hipErrorInvalidValue;
    // the buffer descriptors address one 256-row panel: 32-bit byte offsets
    if ((long long)256 * ldw * 2 >= (1ll << 31) || (long long)256 * 2 * K * 2 >= (1ll << 31)) return hipErrorInvalidValue;
#if RS_DIAG
    if (g_stamps) return launch_gemm_x3s_v<268435456>(epi, A, W, ldw, M_pad, N_pad, K, ep, st);
#endif
    return launch_gemm_x3s_v<0>(epi, A, W, ldw, M_pad, N_pad, K, ep, st);
}

#if RS_DIAG
// Diagnostic entry (not part of the scoring path): on = 1 allocates and zeroes the stamp buffer
// and switches the split-operand GEMM launches to their stamp builds; on = 0 copies the buffer
// (STAMP_WORDS u64: [instance][workgroup][phase], phases 0 K loop, 1 bias + next stage, 2 residual,
// 3 statistics + publish, 4 poll, 5 LN apply, 6 stores, 7 tiles, 8 prologue) to host_out (may be
// null), frees it and switches back.  Call on an idle device.
extern "C" int rs_debug_stamps(int on, unsigned long long* host_out) {
    if (on) {
        if (!g_stamps && hipMalloc((void**)&g_stamps, STAMP_WORDS * 8) != hipSuccess) return -2;
        return hipMemset(g_stamps, 0, STAMP_WORDS * 8) == hipSuccess ? 0 : -2;
    }
    if (!g_stamps) return -1;
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    if (host_out && hipMemcpy(host_out, g_stamps, STAMP_WORDS * 8, hipMemcpyDeviceToHost) != hipSuccess) return -2;
    (void)hipFree(g_stamps);
    g_stamps = nullptr;
    return 0;
}
#endif

hipError_t launch_gemm(int epi, const f16* A, const f16* W, int M_pad, int N_pad, int K,
                       const EpiArgs& ep, hipStream_t st, int tag) {
    if (M_pad % 256 || N_pad % 128 || K % 64 || M_pad <= 0) return hipErrorInvalidValue;
    switch (epi) {
        case EPI_BIAS_F16: return launch_epi<EPI_BIAS_F16>(A, W, M_pad, N_pad, K, ep, st, tag);
        case EPI_GELU_F16: return launch_epi<EPI_GELU_F16>(A, W, M_pad, N_pad, K, ep, st, tag);
        case EPI_GELU_F32: return launch_epi<EPI_GELU_F32>(A, W, M_pad, N_pad, K, ep, st, tag);
        case EPI_RES_F32: return launch_epi<EPI_RES_F32>(A, W, M_pad, N_pad, K, ep, st, tag);
        case EPI_LSE: return launch_epi<EPI_LSE>(A, W, M_pad, N_pad, K, ep, st, tag);
        case EPI_BIAS_F32: return launch_epi<EPI_BIAS_F32>(A, W, M_pad, N_pad, K, ep, st, tag);
        case EPI_RESLN_F32: return launch_epi<EPI_RESLN_F32>(A, W, M_pad, N_pad, K, ep, st, tag);
    }
    return hipErrorInvalidValue;
}

// Timing/diagnostic entry (not part of the scoring path): one GEMM with an explicit tile
// configuration and VAR bits, C = A[M,K].W[N,K]^T + bias -> fp16 [M, N].
extern "C" int rs_debug_gemm(int cfg, int dbg, const void* A, const void* W, const float* bias, void* out,
                             int M, int N, int K, void* stream) {
    EpiArgs ep{};
    ep.bias = bias; ep.out = out; ep.ldc = N; ep.m_valid = M; ep.kx = 1; ep.nlog = N;
    hipStream_t st = (hipStream_t)stream;
    const f16* a = (const f16*)A;
    const f16* w = (const f16*)W;
    hipError_t e = hipErrorInvalidValue;
    if (M % 256 || N % 256 || K % 64) return -1;
    if (cfg == 31 || cfg == 32) {  // split-operand fp16x3 (A [M, 2K], W [N, 2K] interleaved images): 31 GELU image, 32 fp32
        // dbg 0: the production kernel.  The RS_DIAG build adds the timing diagnostics of
        // gemm_x3s_kernel (wrong results; tools/x3s_epi_probe.py): 1 no K-loop staging, 2 no
        // epilogue stores (20 / 52: the same, older probe numbering), 3 neither, 50 DMA never
        // waited for, 51 stores onto row panel 0 (no HBM write burst), 53 both
        ep.nlog = N;
        const int epi = cfg == 31 ? EPI_GELU_F16 : EPI_BIAS_F32;
        if (cfg == 31) ep.ldc = 2 * N;
        if (dbg == 0) e = launch_gemm_x3s(epi, a, w, 2 * K, M, N, K, ep, st);
#if RS_DIAG
#define RS_X3(VAR_)                                                                        \
    (cfg == 31 ? launch_x3s<EPI_GELU_F16, VAR_>(a, w, M, N, K, ep, st) : launch_x3s<EPI_BIAS_F32, VAR_>(a, w, M, N, K, ep, st))
        else switch (dbg) {
            case 1: e = RS_X3(1); break;
            case 2: case 20: case 52: e = RS_X3(2); break;
            case 3: e = RS_X3(3); break;
            case 50: e = RS_X3(8); break;
            case 51: e = RS_X3(33554432); break;
            case 53: e = RS_X3(8 | 33554432); break;
            default: return -1;
        }
#undef RS_X3
#else
        else return -1;
#endif
        return e == hipSuccess ? 0 : -2;
    }
    // fp16 kernels: 9 / 11 persistent bias / GELU with the plain schedule (the bitwise reference
    // of the production schedule), 21 / 18 the production persistent schedules, 0 (dbg 8384) the
    // pipelined kernel with non-temporal stores
    switch (cfg) {
        case 9: e = launch_persist<EPI_BIAS_F16>(a, w, M, N, K, ep, st); break;
        case 11: e = launch_persist<EPI_GELU_F16>(a, w, M, N, K, ep, st); break;
        case 21: e = launch_persist<EPI_BIAS_F16, 786432 | 1048576>(a, w, M, N, K, ep, st); break;
        case 18: e = launch_persist<EPI_GELU_F16, 262144 | 524288>(a, w, M, N, K, ep, st); break;
        case 0:
            if (dbg != 8384) return -1;
            e = launch_t<256, 256, 2, 4, 2, 64, EPI_BIAS_F16, 8384>(a, w, M, N, K, ep, st);
            break;
        default: return -1;
    }
    return e == hipSuccess ? 0 : -2;
}

// Test utility (not part of the scoring path): y[i] = gelu2(x[i]) — the epilogues' GELU evaluated
// elementwise in fp32 (tests/test_gpu_gemm.py checks it against torch's exact-erf GELU).
namespace {
__global__ void __launch_bounds__(256) gelu_eval_kernel(const float* __restrict__ x, float* __restrict__ y, int n) {
    const int i = 2 * (blockIdx.x * 256 + threadIdx.x);
    if (i + 1 < n) {
        const f32x2 v = gelu2((f32x2){x[i], x[i + 1]});
        y[i] = v.x;
        y[i + 1] = v.y;
    } else if (i < n) {
        y[i] = gelu2((f32x2){x[i], 0.f}).x;
    }
}
}  // namespace

extern "C" int rs_debug_gelu(const float* x, float* y, int n, void* stream) {
    if (n <= 0) return n == 0 ? 0 : -1;
    hipLaunchKernelGGL(gelu_eval_kernel, dim3((n + 511) / 512), dim3(256), 0, (hipStream_t)stream, x, y, n);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Test utility (not part of the scoring path): keeps `blocks` workgroups resident for `usec`
// microseconds, one per CU (each declares the whole 160 KiB of LDS), on `stream` — a kernel of
// another stream (or process) holding CUs while the scorer runs.  Bounded by the constant-rate
// s_memrealtime clock (100 MHz): every wave exits once the time is up.  d_out (may be null,
// 3 x blocks ints): [0, blocks) spins, [blocks, 2 blocks) where the workgroup ran (XCC_ID << 24 |
// HW_ID bits 23:0: CU_ID 11:8, SH_ID 12, SE_ID 15:13), [2 blocks, 3 blocks) its start time
// (s_memrealtime, low 32 bits).
namespace {
__global__ void __launch_bounds__(64) occupy_kernel(long long ticks, int* out) {
    extern __shared__ int lds_hold[];
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)\n\ts_getreg_b32 %1, hwreg(HW_REG_XCC_ID)"
                 : "=s"(hw), "=s"(xcc));
    int spins = 0;
    while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
        __builtin_amdgcn_s_sleep(8);
        ++spins;
    }
    lds_hold[threadIdx.x] = spins;
    __syncthreads();
    if (threadIdx.x == 0 && out) {                                 // vector stores
        out[blockIdx.x] = lds_hold[0];
        out[gridDim.x + blockIdx.x] = (int)(((xcc & 15u) << 24) | (hw & 0xffffffu));
        out[2 * gridDim.x + blockIdx.x] = (int)(unsigned)t0;
    }
}
}  // namespace

extern "C" int rs_debug_occupy(int blocks, int usec, int* d_out, void* stream) {
    if (blocks <= 0 || blocks > 1365 || usec <= 0 || usec > 5000000) return -1;
    constexpr int smem = 160 * 1024;
    static std::atomic<unsigned> attr_devs{0};
    if (smem_attr_once((const void*)occupy_kernel, smem, attr_devs) != hipSuccess) return -2;
    hipLaunchKernelGGL(occupy_kernel, dim3(blocks), dim3(64), smem, (hipStream_t)stream, (long long)usec * 100, d_out);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
