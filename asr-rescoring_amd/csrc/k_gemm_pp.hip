// Split-operand fp16x3 GEMM with the epilogue overlapped ("ping-pong"): C = A . W^T (+ bias /
// GELU), the fp32-accurate projection of the fp16x3 mode (three fp16 products from two-part
// images, as gemm_x3s_kernel in k_gemm.hip), for the BERT projections without a residual
// (fused QKV :154-156 and BertIntermediate :325-337 of transformers modeling_bert.py).
//
// Why: with one 256x256 tile per workgroup, all eight waves reach their epilogue together, the
// MFMA pipes of the CU idle while it runs, and since every CU does the same at the same time the
// epilogue stores leave the chip as one burst per round of tiles (64 MB at K = 768; round 3:
// 13-18 % of the kernel, profiles/r3w_x3s_stagger_dma.txt prod vs noepi).
//
// Structure: the 8-wave workgroup is two independent 4-wave halves (h = wave >> 2: one wave of
// each half on every SIMD), each walking its own sequence of 128 x 256 tiles (wave tile 128 x 64,
// v_mfma_f32_16x16x32_f16, 96 MFMAs per wave per BK = 32 step).  Half 1 runs D intervals behind
// half 0, about half a tile, so while one half runs its epilogue the other half's K loop has the
// SIMDs' MFMA pipes to itself, and the chip's epilogue stores spread over twice as many, half as
// large bursts.  The halves share one workgroup barrier per INTERVAL (a K step of a half, or one
// of the E chunks its epilogue is cut into); each half pads with bare barriers where it has no
// work, so both execute the same barrier count.
//   * A (the 128-row panel, shared by the half's 4 waves) goes HBM -> LDS by LDS-DMA
//     (buffer_load_dwordx4 ... lds, 16 KiB per half-step into that half's 2-stage ring), one K step
//     ahead;
//   * W (each wave's own 64 columns: no sharing inside a half, none across the phase-shifted
//     halves) goes straight to registers (buffer_load_dwordx4, 8 per wave per step, double
//     buffered, one step ahead) — no LDS traffic for W;
//   * epilogue through the wave-private 4 KiB slabs (as gemm_x3s_kernel): bias (+ GELU), the
//     fp32 output or the two-part image, 16-B non-temporal row stores.
// LDS: 2 halves x 2 stages x 16 KiB + 32 KiB of slabs = 96 KiB.
#include "common.h"
#include "gemm_dev.h"

#include <atomic>
#include <type_traits>
#include <stdlib.h>
#include <string.h>

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int PP_E = 4;            // epilogue intervals per tile

// DV: timing diagnostics (wrong results; rs_debug_gemm dbg 61..): 1 no epilogue stores, 2 halves
// in phase (D = 0), 4 no W loads (stale W registers), 8 no A DMA (stale LDS)
template <int EPI, int DV = 0>
__global__ void __launch_bounds__(512)
gemm_pp_kernel(const f16* __restrict__ A, const f16* __restrict__ W, int K, int ldw, int n_tiles_n, int n_tiles,
               EpiArgs ep) {
    static_assert(EPI == EPI_BIAS_F32 || EPI == EPI_GELU_F16, "pp epilogues: fp32 out, two-part GELU image");
    constexpr int BM = 128, BK = 32, RB = 64;          // half tile 128 x 256; 64-B LDS rows
    constexpr int PART = BM * RB;                       // 8 KiB: hi or lo part of a half's stage
    constexpr int STAGE = 2 * PART;                     // 16 KiB
    constexpr int E = PP_E;
    extern __shared__ __attribute__((aligned(16))) char smem[];          // [half][stage][part][row][64 B]
    __shared__ __attribute__((aligned(16))) char slabs[8 * 4096];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int h = wave >> 2, wn = wave & 3;
    const int r16 = lane & 15, q4 = lane >> 4;
    const int nk = K / BK;
    const int P = nk + E;                               // intervals per tile (nk even: P even)
    const int D = (DV & 2) ? 0 : (P / 2) & ~1;          // half 1's lag (even: W register parity)

    // ---- tile sequence of this half: grouped-order indices 2 wg + h, + 2 G, ... -----------
    const int G = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, pos = bid >> 3, qg = G >> 3, rg = G & 7;
    const int wg = (xcd < rg ? xcd * (qg + 1) : rg * (qg + 1) + (xcd - rg) * qg) + pos;
    const int stride = 2 * G;
    auto count = [&](int f) { return f < n_tiles ? (n_tiles - f + stride - 1) / stride : 0; };
    const int T0 = count(2 * wg), T1 = count(2 * wg + 1);
    if (T0 == 0) return;                                // (the launch sizes the grid so this never happens)
    const int Tm = h ? T1 : T0;
    const int pre = h ? D : 0;
    const int total = max(T0 * P, T1 > 0 ? D + T1 * P : 0);
    const int n_tiles_m = n_tiles / n_tiles_n;
    auto tile_of = [&](int i, int& m0, int& n0) {      // i-th tile of this half
        const int idx = 2 * wg + h + i * stride;
        const int GM = ep.group_m, per_group = GM * n_tiles_n;
        const int g = idx / per_group, loc = idx - g * per_group;
        const int gm = min(GM, n_tiles_m - g * GM);
        const int tn = loc / gm;
        m0 = (g * GM + (loc - tn * gm)) * BM;
        n0 = tn * 256;
    };

    // ---- staging: A pieces (LDS-DMA) and W fragments (registers) -------------------------
    // piece p (0..3) of wave wn: part p & 1, rows 16 (wn + 4 (p >> 1)) + lane / 4, 16-B chunk
    // lane & 3 of the LDS row holds source chunk (lane & 3) ^ g16(row >> 2)
    const int ring_off = h * 2 * STAGE;
    char* ring = smem + ring_off;
    const size_t ld2 = (size_t)2 * K;
    // one lane offset per operand; the piece / fragment part of the address is wave-uniform and
    // rides the scalar offset (row >> 2 & 3 = lane >> 4 for every piece: rows 16-aligned)
    const int voffA = ((lane >> 2) * (int)ld2 + (((lane & 3) ^ g16(lane >> 4)) << 3)) * 2;
    auto soffA = [&](int p) { return (16 * (wn + 4 * (p >> 1)) * (int)ld2 + (p & 1) * K) * 2; };
    // W fragment j (column block 16 j of the wave's 64), part pr: lane l reads W row
    // n0 + 64 wn + 16 j + (l & 15) at k-chunk l >> 4 (16 B)
    const int voffW = ((64 * wn + r16) * ldw + 8 * q4) * 2;
    auto soffW = [&](int j, int pr) { return (16 * j * ldw + pr * K) * 2; };
    __amdgpu_buffer_rsrc_t rsA, rsW;
    auto set_rsrc = [&](int m0, int n0) {
        rsA = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (size_t)m0 * ld2), (short)0, (int)(BM * ld2 * 2), 0x00020000);
        rsW = __builtin_amdgcn_make_buffer_rsrc((void*)(W + (size_t)n0 * ldw), (short)0, 256 * ldw * 2, 0x00020000);
    };
    auto piece = [&](int buf, int k0, int p) {
        if constexpr ((DV & 8) != 0) return;
        auto* dst = (__attribute__((address_space(3))) void*)(smem + ring_off + buf * STAGE + (p & 1) * PART +
                                                               (wn + 4 * (p >> 1)) * 1024);
        const int so = soffA(p) + k0 * 2;             // (a call in the builtin's argument list
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, dst, 16, voffA, so, 0, 0);   //  drops the host stub)
    };
    u32x4 wb[2][4][2];                                  // [register buffer][j][hi, lo]
    auto wload = [&](u32x4 (&w)[4][2], int k0) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int pr = 0; pr < 2; ++pr) w[j][pr] = __builtin_amdgcn_raw_buffer_load_b128(rsW, voffW, soffW(j, pr) + k0 * 2, 0);
    };

    f32x4 acc16[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc16[i][j] = (f32x4)(0.f);
    const half8 down = (half8)(f16)X3_DOWN;
    const int offA16 = r16 * RB + ((q4 ^ g16(r16 >> 2)) << 4);

    // one K step: 96 MFMAs over the A stage `buf` and the W registers w, row block by row block
    // (12 MFMAs each: the three products x 4 column blocks), the next row block's two fragments
    // read while the current one computes — 128 accumulators + 64 W registers + 16 A registers fit
    // the 256 of two waves per SIMD.  The next step's four A pieces (into `nbuf`) and eight W loads
    // (into wnext) ride the first four row blocks.
    auto kstep = [&](int buf, u32x4 (&w)[4][2], int nbuf, int k0n, u32x4 (&wnext)[4][2], bool a_next) {
        const char* sb = ring + buf * STAGE;
        half8 ah[2], al[2];
        auto read_a = [&](int ib, half8& h_, half8& l_) {
            h_ = *(const half8*)(sb + offA16 + ib * 1024);
            l_ = *(const half8*)(sb + PART + offA16 + ib * 1024);
        };
        read_a(0, ah[0], al[0]);
#pragma unroll
        for (int ib = 0; ib < 8; ++ib) {
            half8& a = ah[ib & 1];
            half8& l = al[ib & 1];
            if (ib + 1 < 8) read_a(ib + 1, ah[(ib + 1) & 1], al[(ib + 1) & 1]);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc16[ib][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, w[j][0]), a, acc16[ib][j], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc16[ib][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, w[j][0]) * down, l, acc16[ib][j],
                                                                      0, 0, 0);
            const half8 ad = a * down;                  // A_hi / 64
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc16[ib][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(half8, w[j][1]), ad, acc16[ib][j], 0, 0, 0);
            if (ib < 4) {
                __builtin_amdgcn_sched_barrier(0);
                if (a_next) piece(nbuf, k0n, ib);
                if constexpr ((DV & 4) == 0) {
                    wnext[ib][0] = __builtin_amdgcn_raw_buffer_load_b128(rsW, voffW, soffW(ib, 0) + k0n * 2, 0);
                    wnext[ib][1] = __builtin_amdgcn_raw_buffer_load_b128(rsW, voffW, soffW(ib, 1) + k0n * 2, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    };

    // ---- epilogue chunk e (rows 32 e .. 32 e + 31 of the wave's 128): bias (+ GELU), slab pass,
    // 16-B non-temporal stores
    f32x4 bq[4];
    char* slb = slabs + wave * 4096;
    const int rr0 = lane >> 3, c16 = lane & 7;
    auto epi_chunk = [&](auto ec, int cm0, int cn0) {
        constexpr int e = decltype(ec)::value;          // compile-time: acc16 stays in registers
        if constexpr ((DV & 1) != 0) {
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc16[2 * e + a][j]));
            return;
        }
        if (e == 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float* bp = ep.bias + cn0 + 64 * wn + 16 * j + 4 * q4;
                asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(bq[j]) : "v"(bp) : "memory");
            }
            asm volatile("s_waitcnt vmcnt(0)" : "+v"(bq[0]), "+v"(bq[1]), "+v"(bq[2]), "+v"(bq[3]) : : "memory");
        }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int q = 0; q < 4; q += 2) {
                    f32x2 v = {acc16[2 * e + a][j][q] + bq[j][q], acc16[2 * e + a][j][q + 1] + bq[j][q + 1]};
                    if constexpr (EPI == EPI_GELU_F16) v = gelu2(v);
                    acc16[2 * e + a][j][q] = v.x;
                    acc16[2 * e + a][j][q + 1] = v.y;
                }
        if constexpr (EPI == EPI_BIAS_F32) {
            // two 32 x 32 fp32 slab blocks: column blocks 2 j2 + b
#pragma unroll
            for (int j2 = 0; j2 < 2; ++j2) {
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int b = 0; b < 2; ++b) {
                        const int row = 16 * a + r16, ch = 4 * b + q4;
                        *(f32x4*)(slb + row * 128 + ((ch ^ (row & 7)) << 4)) = acc16[2 * e + a][2 * j2 + b];
                    }
                float* ob = (float*)ep.out + (size_t)(cm0 + 32 * e) * ep.ldc + cn0 + 64 * wn + 32 * j2 + 4 * c16;
                uint4 v[4];
                slab_read4(slb, rr0, c16, v);
#pragma unroll
                for (int it = 0; it < 4; ++it) st16<64>((uint4*)(ob + (size_t)(it * 8 + rr0) * ep.ldc), v[it]);
            }
        } else {
            // two-part image (hi, lo * 64) of the 32 x 64 block, nlog columns apart
#pragma unroll
            for (int img = 0; img < 2; ++img) {
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        half4 hv;
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const float x = acc16[2 * e + a][j][q];
                            const f16 hi = (f16)x;
                            hv[q] = img == 0 ? hi : x3_lo(x, hi);
                        }
                        const int row = 16 * a + r16, byte = 32 * j + 8 * q4;
                        *(half4*)(slb + row * 128 + (((byte >> 4) ^ (row & 7)) << 4) + (byte & 8)) = hv;
                    }
                f16* ob = (f16*)ep.out + (size_t)(cm0 + 32 * e) * ep.ldc + img * ep.nlog + cn0 + 64 * wn + 8 * c16;
                uint4 v[4];
                slab_read4(slb, rr0, c16, v);
#pragma unroll
                for (int it = 0; it < 4; ++it) st16<64>((uint4*)(ob + (size_t)(it * 8 + rr0) * ep.ldc), v[it]);
            }
        }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc16[2 * e + a][j] = (f32x4)(0.f);    // the next tile starts at 0
    };

    // ---- the interval sequence of this half: [pre pads][tile: nk K steps, E epilogue chunks]...
    // [post pads]; every interval is one workgroup barrier (the two halves run different code
    // between barriers: s_barrier counts waves, not program counters)
    if (h) {
        for (int i = 0; i < pre; ++i) asm volatile("s_barrier" ::: "memory");
    }
    int m0 = 0, n0 = 0;
    if (Tm > 0) {
        tile_of(0, m0, n0);
        set_rsrc(m0, n0);
#pragma unroll
        for (int p = 0; p < 4; ++p) piece(0, 0, p);
        wload(wb[0], 0);
    }
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    for (int ti = 0; ti < Tm; ++ti) {
        const int cm0 = m0, cn0 = n0;
        // K step kt (buffer / W registers kt & 1): landed for this wave — after an epilogue, stage
        // 0 and W(0) are older than its 32 stores (the bias loads were waited for) — then the barrier
        auto step = [&](auto parc, int kt) {
            constexpr int PAR = decltype(parc)::value;
            if (kt == 0 && ti > 0) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("s_barrier" ::: "memory");
            bool a_next = true;
            int k0n = (kt + 1) * BK;
            if (kt + 1 == nk) {                         // the next tile's stage 0 + W(0)
                if (ti + 1 < Tm) {
                    tile_of(ti + 1, m0, n0);
                    set_rsrc(m0, n0);
                    k0n = 0;
                } else {
                    a_next = false;
                    k0n = 1 << 28;                      // past the W panel: the loads return 0
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            kstep(PAR, wb[PAR], PAR ^ 1, k0n, wb[PAR ^ 1], a_next);
            __builtin_amdgcn_sched_barrier(0);
        };
        for (int kt = 0; kt < nk; kt += 2) {
            step(I0(), kt);
            step(I1(), kt + 1);
        }
        static_assert(E == 4, "epilogue chunks");
        asm volatile("s_barrier" ::: "memory");
        epi_chunk(std::integral_constant<int, 0>(), cm0, cn0);
        asm volatile("s_barrier" ::: "memory");
        epi_chunk(std::integral_constant<int, 1>(), cm0, cn0);
        asm volatile("s_barrier" ::: "memory");
        epi_chunk(std::integral_constant<int, 2>(), cm0, cn0);
        asm volatile("s_barrier" ::: "memory");
        epi_chunk(std::integral_constant<int, 3>(), cm0, cn0);
    }
    for (int i = pre + Tm * P; i < total; ++i) asm volatile("s_barrier" ::: "memory");
}

int n_cus_pp() {
    static int n = [] {
        int dev = 0, v = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
        return v > 0 ? v : 256;
    }();
    return n;
}

template <int EPI, int DV = 0>
hipError_t launch_pp(const f16* A, const f16* W, int ldw, int M_pad, int N_pad, int K, const EpiArgs& ep, hipStream_t st) {
    constexpr int smem = 4 * 16384;                     // A rings (2 halves x 2 stages); + 32 KiB slabs
    if (K % 64 || K < 64 || M_pad % 256 || N_pad % 256 || ldw < 2 * K) return hipErrorInvalidValue;
    if ((long long)256 * ldw * 2 >= (1ll << 31) || (long long)128 * 2 * K * 2 >= (1ll << 31)) return hipErrorInvalidValue;
    static std::atomic<unsigned> attr_devs{0};
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev)) return e;
    const unsigned bit = 1u << (dev & 31);
    if (!(attr_devs.load(std::memory_order_acquire) & bit)) {
        if (hipError_t e = hipFuncSetAttribute((const void*)gemm_pp_kernel<EPI, DV>, hipFuncAttributeMaxDynamicSharedMemorySize, smem))
            return e;
        attr_devs.fetch_or(bit, std::memory_order_release);
    }
    const int ntn = N_pad / 256, n_tiles = (M_pad / 128) * ntn;
    const int cus = n_cus_pp() / 8 * 8;
    const int grid = std::min(cus, (n_tiles + 1) / 2);
    static const int gm_env = getenv("RS_PP_GROUP_M") ? atoi(getenv("RS_PP_GROUP_M")) : 0;
    EpiArgs e2 = ep;
    e2.group_m = gm_env > 0 ? gm_env : 16;              // 128-row panels per group
    hipLaunchKernelGGL((gemm_pp_kernel<EPI, DV>), dim3(grid), dim3(512), smem, st, A, W, K, ldw, ntn, n_tiles, e2);
    return hipGetLastError();
}

}  // namespace

// Split-operand GEMM with the epilogue overlapped (see top): EPI_BIAS_F32 or EPI_GELU_F16; the
// same operands and contract as launch_gemm_x3s.
hipError_t launch_gemm_pp(int epi, const f16* A, const f16* W, int ldw, int M_pad, int N_pad, int K, const EpiArgs& ep,
                          hipStream_t st, int dv) {
    if (epi == EPI_BIAS_F32) {
        switch (dv) {
            case 1: return launch_pp<EPI_BIAS_F32, 1>(A, W, ldw, M_pad, N_pad, K, ep, st);
            case 2: return launch_pp<EPI_BIAS_F32, 2>(A, W, ldw, M_pad, N_pad, K, ep, st);
            case 3: return launch_pp<EPI_BIAS_F32, 3>(A, W, ldw, M_pad, N_pad, K, ep, st);
            case 4: return launch_pp<EPI_BIAS_F32, 4>(A, W, ldw, M_pad, N_pad, K, ep, st);
            case 5: return launch_pp<EPI_BIAS_F32, 5>(A, W, ldw, M_pad, N_pad, K, ep, st);
            case 13: return launch_pp<EPI_BIAS_F32, 13>(A, W, ldw, M_pad, N_pad, K, ep, st);
            default: break;
        }
    }
    switch (epi) {
        case EPI_BIAS_F32: return launch_pp<EPI_BIAS_F32>(A, W, ldw, M_pad, N_pad, K, ep, st);
        case EPI_GELU_F16: return launch_pp<EPI_GELU_F16>(A, W, ldw, M_pad, N_pad, K, ep, st);
    }
    return hipErrorInvalidValue;
}
