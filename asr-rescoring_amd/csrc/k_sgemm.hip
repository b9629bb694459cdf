// fp32 GEMMs of the trainer: the forward projections, the input
// gradients and the weight gradients of every nn.Linear the reference trains
// (RescoreBert/main.py:104-150, MLM_PLL/main.py:89-97 through transformers' BertModel).
//
// The reference trains in fp32, so these run on the f32-input MFMA (v_mfma_f32_32x32x2_f32:
// exact f32, every result a k-ordered fmaf chain) rather than on the fp16 split-operand
// kernels of the scoring path.  C[m][n] = sum_k A(m, k) B(n, k); each operand is read either
// with k contiguous ("KC": [row][ld]) or with its output dimension contiguous ("MC":
// [k][ld]), which covers the three forms a Linear needs:
//   forward  Y  = X  · Wᵀ   A = X  (KC)   B = W  (KC)
//   dgrad    dX = dY · W    A = dY (KC)   B = W  (MC: W[n][k'] read with k' = output column)
//   wgrad    dW = dYᵀ· X    A = dY (MC)   B = X  (MC)
//
// Tiles (by shape, sg_pick's time model): 128×128 (4 waves of 64×64) or 192×128 (4 waves of
// 96×64), two workgroups per CU, or for the ~1k-token GEMMs the 64×64 direct-to-register form
// (sgemm_d64_kernel, below; other tiles are A/B knobs); BK = 32; two LDS stages filled by LDS-DMA
// (buffer_load_dwordx4 … lds, 1 KiB per wave-instruction) with one barrier per K-step and two
// waves per SIMD.  No register staging and no transposing LDS writes: the DMA writes each
// operand's natural image —
//   KC: [row][32 k] rows of 128 B, 16-B chunks XOR-swizzled by (row >> 1) & 7 on the source
//       address, so a wave's ds_read_b128 of 16 rows × one chunk hits 64 distinct banks;
//   MC: [k][R rows] rows of 4R bytes (fragment reads are ds_read_b32 of 32 consecutive rows).
// The K index inside a K-step is permuted (A and B alike, so the product is unchanged):
// MFMA step kk of lane half h takes k = 16h + kk, which makes a KC lane's 16 values of a
// K-step 64 contiguous bytes (4 × ds_read_b128).  All of a K-step's fragments are read into
// registers before the next K-step's DMA is issued, so no LDS read follows an in-flight DMA
// into the same LDS object (the compiler would wait vmcnt(0) before it).
// Few output tiles (the weight gradients of a ~1k-token batch, the projections of a small
// batch) are split over K: each split writes its partial tile to a workspace and an ordered
// sum over the splits closes it — no float atomics, so a training step stays bitwise
// reproducible.  Edges: lanes whose row or k lies outside the operand load from an offset past
// the buffer descriptor's extent, which the hardware returns as zeros.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "train.h"

namespace {

typedef float f32x16_t __attribute__((ext_vector_type(16)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t sg_rsrc(const float* p, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
}

// Workgroup -> (split z, output tile) with an XCD-aware bijective remap (MI355X_MICROARCH:
// blocks b and b + 8 share an XCD): each XCD takes a contiguous range of the work list, and
// inside a split the tiles go in groups of 8 row panels walked column by column, so the
// ~64 workgroups an XCD runs at once share 8 A panels and 8 B panels in its L2 instead of
// touching every panel of the operands (the row-major grid dealt every tile row's column
// tiles to all eight XCDs).
__device__ __forceinline__ void sg_tile(int tiles_m, int tiles_n, int& tm, int& tn, int& z) {
    const int nwg = gridDim.x, b = blockIdx.x;
    const int xcd = b & 7, pos = b >> 3, q = nwg >> 3, r = nwg & 7;
    const int w = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
    const int per = tiles_m * tiles_n;
    z = w / per;
    const int t = w - z * per;
    constexpr int GM = 8;
    const int g = t / (GM * tiles_n), loc = t - g * GM * tiles_n;
    const int gm = min(GM, tiles_m - g * GM);
    tn = loc / gm;
    tm = g * GM + (loc - tn * gm);
}

// One operand's image of R rows × BK: its DMA source for this wave's pieces of a K-step (1 KiB
// each; NP of them) and its fragment reads.  rows: operand rows (M or N) in [0, rows); k in
// [kb, ke).  KC image: [R][BK] floats (rows of 4 BK bytes = NCH 16-B chunks), chunk c of row r
// stored at position c ^ ((r >> SH) & (NCH - 1)) (SH: log2 of the rows per 256-B bank row), so
// the ds_read_b128 of 16 rows × one chunk hits 64 distinct banks; MC image: [BK][R] floats.
template <bool KC, int R, int NW, int BK>
struct SgOperand {
    static constexpr int NP = R * BK * 4 / 1024 / NW;        // pieces per wave per K-step
    static constexpr int NCH = BK / 4, RP = 1024 / (BK * 4), SH = BK == 32 ? 1 : 2;
    static_assert(BK == 16 || BK == 32, "BK");
    static_assert(NP >= 1 && NP * NW * 1024 == R * BK * 4, "pieces must split evenly over the waves");
    __amdgpu_buffer_rsrc_t rs;
    unsigned oob;                // an offset past the descriptor's extent: loads return 0
    unsigned voff[NP];           // per piece: byte offset of this lane's 16 B at k0 = 0 (oob: row outside)
    int krow[NP];                // KC: the lane's k within the step (4 lc); MC: its k-row
    int ld;

    __device__ void init(const float* src, int ld_, int rows, int row0, int wave, int lane) {
        ld = ld_;
        oob = 0x7FFFFFF0u;       // the operand's extent is host-checked below 2^31 bytes
        rs = sg_rsrc(src, oob);
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            const int p = NW * i + wave;
            if (KC) {
                const int r = RP * p + lane / NCH;                          // image row of this lane
                const int lc = (lane % NCH) ^ ((r >> SH) & (NCH - 1));      // logical 16-B chunk
                krow[i] = 4 * lc;
                voff[i] = row0 + r < rows ? (unsigned)(((row0 + r) * ld + 4 * lc) * 4) : oob;
            } else {
                const int byte = p * 1024 + lane * 16;
                const int kr = byte / (R * 4), c = row0 + (byte % (R * 4)) / 4;
                krow[i] = kr;
                voff[i] = c < rows ? (unsigned)((kr * ld + c) * 4) : oob;
            }
        }
    }
    // DMA this wave's pieces of K-step k0 into the image at lds.  The lane offsets are fixed
    // per workgroup (k0 rides in the scalar offset), so each piece's offset stays in its own
    // register across the loop and the DMAs issue back to back (an offset re-formed per piece
    // in one reused VGPR makes every v_cndmask wait for the previous buffer_load to read it).
    // Only a K-step that crosses ke (the tail of K) masks lanes per step.  (The builtin's
    // arguments are plain locals on purpose: with a conditional expression or an array element
    // written in place as the offset argument, hipcc / ROCm 7.2 silently emitted no host launch
    // stub for the MC instantiations — an undefined symbol at load time.)
    __device__ __forceinline__ void stage(char* lds, int wave, int k0, int ke) const {
        const int so = KC ? k0 * 4 : k0 * ld * 4;
        if (k0 + BK <= ke) {                     // wave-uniform: every K-step but the tail
#pragma unroll
            for (int i = 0; i < NP; ++i) {
                const unsigned vo = voff[i];
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rs, (__attribute__((address_space(3))) void*)(lds + (NW * i + wave) * 1024), 16, vo, so, 0, 0);
            }
        } else {
#pragma unroll
            for (int i = 0; i < NP; ++i) {
                const bool in = k0 + krow[i] < ke;
                const unsigned vo = in ? voff[i] : oob;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rs, (__attribute__((address_space(3))) void*)(lds + (NW * i + wave) * 1024), 16, vo, so, 0, 0);
            }
        }
    }
    // piece i of stage() without the wave-uniform branch: masked by its own k (only a tail K-step
    // has masked lanes), so the DMA pieces can sit inside a straight-line MFMA stream
    __device__ __forceinline__ void stage_piece(char* lds, int wave, int k0, int ke, int i) const {
        const int so = KC ? k0 * 4 : k0 * ld * 4;
        const bool in = k0 + krow[i] < ke;
        const unsigned vo = in ? voff[i] : oob;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs, (__attribute__((address_space(3))) void*)(lds + (NW * i + wave) * 1024), 16, vo, so, 0, 0);
    }
    // The fragment reads of T 32-row tiles (rows r0 + 32 t) cut into units the software-pipelined
    // kernel spreads over its MFMA stream: KC, unit u = one ds_read_b128 (tile u / 4, 16-B chunk
    // u % 4); MC, unit u = k-row u of every tile (adjacent tiles pair into ds_read2_b32).
    static constexpr int units(int tiles) { return KC ? 4 * tiles : BK / 2; }
    template <int T>
    __device__ __forceinline__ static void frag_unit(const char* img, int r0, int h, int u, float (&f)[T][BK / 2]) {
        if (KC) {
            const int t = u / 4, q = u % 4, r = r0 + 32 * t;
            const int pc = ((BK / 8) * h + q) ^ ((r >> SH) & (NCH - 1));
            const float4 v = *(const float4*)(img + r * BK * 4 + pc * 16);
            f[t][4 * q] = v.x; f[t][4 * q + 1] = v.y; f[t][4 * q + 2] = v.z; f[t][4 * q + 3] = v.w;
        } else {
#pragma unroll
            for (int t = 0; t < T; ++t) f[t][u] = *(const float*)(img + ((BK / 2) * h + u) * R * 4 + (r0 + 32 * t) * 4);
        }
    }
    // fragments of one 32-row MFMA tile for a K-step: f[kk] = operand(row r, k = (BK/2) h + kk)
    __device__ __forceinline__ static void frag(const char* img, int r, int h, float (&f)[BK / 2]) {
        if (KC) {
#pragma unroll
            for (int q = 0; q < BK / 8; ++q) {
                const int pc = ((BK / 8) * h + q) ^ ((r >> SH) & (NCH - 1));
                const float4 v = *(const float4*)(img + r * BK * 4 + pc * 16);
                f[4 * q] = v.x; f[4 * q + 1] = v.y; f[4 * q + 2] = v.z; f[4 * q + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int kk = 0; kk < BK / 2; ++kk) f[kk] = *(const float*)(img + ((BK / 2) * h + kk) * R * 4 + r * 4);
        }
    }
};

// C[M][N] (+)= A·B over k in [z·kc, min(K, (z+1)·kc)) for split z (sg_tile).
// ws == nullptr: C = acc (+ C when accum).  Otherwise the partial goes to ws[z][M][N].
// Tile BM × BN × BK, waves of TM × 64 (TM/32 × 2 MFMA tiles of 32×32), OCC workgroups per CU.
template <bool AKC, bool BKC, int BM, int BN, int TM, int BK, int OCC>
__global__ void __launch_bounds__((BM / TM) * (BN / 64) * 64, OCC * (BM / TM) * (BN / 64) / 4)
sgemm_dma_kernel(const float* __restrict__ A, int lda, const float* __restrict__ B, int ldb, float* __restrict__ C,
                 int ldc, int M, int N, int K, int kc, int accum, float* __restrict__ ws) {
    constexpr int WM = BM / TM, WN = BN / 64, NW = WM * WN, MT = TM / 32, HK = BK / 2;
    constexpr int IMG_A = BM * BK * 4, STAGE = (BM + BN) * BK * 4;
    using OA = SgOperand<AKC, BM, NW, BK>;
    using OB = SgOperand<BKC, BN, NW, BK>;
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int tm, tn, z;
    sg_tile((M + BM - 1) / BM, (N + BN - 1) / BN, tm, tn, z);
    const int m0 = tm * BM, n0 = tn * BN;
    const int kb = z * kc, ke = min(K, kb + kc);
    const int wm = (wave % WM) * TM, wn = (wave / WM) * 64;
    const int h = lane >> 5, c = lane & 31;

    OA oa;
    OB ob;
    oa.init(A, lda, M, m0, wave, lane);
    ob.init(B, ldb, N, n0, wave, lane);

    f32x16_t acc[MT][2];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    oa.stage(smem, wave, kb, ke);
    ob.stage(smem + IMG_A, wave, kb, ke);
    int buf = 0;
    for (int k0 = kb; k0 < ke; k0 += BK) {
        // this K-step landed for this wave; the barrier: for every wave, and every wave is done
        // reading the other buffer (its fragments of the previous step are in registers)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const char* st = smem + buf * STAGE;
        float fa[MT][HK], fb[2][HK];
#pragma unroll
        for (int i = 0; i < MT; ++i) OA::frag(st, wm + 32 * i + c, h, fa[i]);
#pragma unroll
        for (int j = 0; j < 2; ++j) OB::frag(st + IMG_A, wn + 32 * j + c, h, fb[j]);
        // fragments in registers before the next K-step's DMA goes into the other buffer
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        if (k0 + BK < ke) {
            char* nx = smem + (buf ^ 1) * STAGE;
            oa.stage(nx, wave, k0 + BK, ke);
            ob.stage(nx + IMG_A, wave, k0 + BK, ke);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kk = 0; kk < HK; ++kk)
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][kk], fb[j][kk], acc[i][j], 0, 0, 0);
        buf ^= 1;
    }

    // D map of the 32x32 forms: column = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    float* P = ws ? ws + (size_t)z * M * N : nullptr;
#pragma unroll
    for (int i = 0; i < MT; ++i)
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

// Software-pipelined form with a straight-line K loop (cfg 12, 17, 18).  The form above reads a
// K-step's fragments between the barrier and its MFMAs, so every wave of a CU reads its 16 KiB
// from LDS at the same moment while its MFMA pipe idles: at one workgroup per CU (a 5.3k-token
// GEMM with N = 768 has 252 tiles of 128×128) that is ≈ 20 % of each K-step.  Here the
// fragments of step t + 1 are read during step t's MFMAs, spread over its first 12 kk groups,
// the DMA pieces of step t + NS over its first 8, and the only gap left between two MFMA
// streams is the barrier.  NS LDS stages in NS distinct __shared__ objects (the compiler then
// sees that the DMA into one does not alias the fragment reads from another and puts no
// vmcnt(0) in front of them), step s in stage s % NS: step t, from the barrier on, issues the
// DMA of step t + NS into the stage step t came from (its fragments are in registers, every
// wave's reads completed before the barrier), so each DMA has NS - 1 K-steps to land.  Two
// register sets of fragments swap roles from step to step; a loop trip is lcm(2, NS) steps so
// every stage and register role is a compile-time constant, and nothing in a trip branches (a
// DMA past the last K-step re-loads the last one), which keeps the accumulators in place.
template <bool AKC, bool BKC, int BM, int BN, int TM, int NS, int OCC>
__global__ void __launch_bounds__((BM / TM) * (BN / 64) * 64, OCC * (BM / TM) * (BN / 64) / 4)
sgemm_sp_kernel(const float* __restrict__ A, int lda, const float* __restrict__ B, int ldb, float* __restrict__ C,
                int ldc, int M, int N, int K, int kc, int accum, float* __restrict__ ws) {
    constexpr int BK = 32, WM = BM / TM, WN = BN / 64, NW = WM * WN, MT = TM / 32, HK = BK / 2;
    constexpr int IMG_A = BM * BK * 4, STAGE = (BM + BN) * BK * 4;
    using OA = SgOperand<AKC, BM, NW, BK>;
    using OB = SgOperand<BKC, BN, NW, BK>;
    constexpr int UA = OA::units(MT), UB = OB::units(2), RG = 12;   // read units over RG kk groups,
    constexpr int NPC = OA::NP + OB::NP < 8 ? OA::NP + OB::NP : 8;  // DMA pieces over NPC kk groups
    static_assert(NS >= 2 && NS <= 4, "stages");
    constexpr int TRIP = NS == 3 ? 6 : NS;                          // steps per loop trip: even, NS | TRIP
    constexpr int NPW = OA::NP + OB::NP;                            // DMA pieces per wave per K-step
    __shared__ __attribute__((aligned(16))) char s0[STAGE];
    __shared__ __attribute__((aligned(16))) char s1[STAGE];
    __shared__ __attribute__((aligned(16))) char s2[NS > 2 ? STAGE : 16];
    __shared__ __attribute__((aligned(16))) char s3[NS > 3 ? STAGE : 16];
    auto stg = [&](int i) -> char* { return i == 0 ? s0 : i == 1 ? s1 : i == 2 ? s2 : s3; };   // i constant
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int tm, tn, z;
    sg_tile((M + BM - 1) / BM, (N + BN - 1) / BN, tm, tn, z);
    const int m0 = tm * BM, n0 = tn * BN;
    const int kb = z * kc, ke = min(K, kb + kc);
    const int nt = (ke - kb + BK - 1) / BK;
    const int wm = (wave % WM) * TM, wn = (wave / WM) * 64;
    const int h = lane >> 5, c = lane & 31;

    OA oa;
    OB ob;
    oa.init(A, lda, M, m0, wave, lane);
    ob.init(B, ldb, N, n0, wave, lane);

    f32x16_t acc[MT][2];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // DMA piece p (A's, then B's) of K-step s (past the last: the last again)
    auto dma_piece = [&](char* dst, int s, int p) {
        const int k0 = kb + min(s, nt - 1) * BK;
        if (p < OA::NP) oa.stage_piece(dst, wave, k0, ke, p);
        else ob.stage_piece(dst + IMG_A, wave, k0, ke, p - OA::NP);
    };
    auto dma = [&](char* dst, int s) {
#pragma unroll
        for (int p = 0; p < OA::NP + OB::NP; ++p) dma_piece(dst, s, p);
    };
    auto mfmas = [&](int kk, const float (&xa)[MT][HK], const float (&xb)[2][HK]) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[i][kk], xb[j][kk], acc[i][j], 0, 0, 0);
    };
    // step t: MFMAs on (xa, xb) = its fragments; (ya, yb) <- step t + 1's from src; DMA of step
    // t + 2 into dst (= the stage step t was read from)
    auto step = [&](int t, char* dst, const char* src, const float (&xa)[MT][HK], const float (&xb)[2][HK],
                    float (&ya)[MT][HK], float (&yb)[2][HK]) {
        // step t + 1's DMA landed (the NS - 2 later ones may still fly); step t's reads done
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"((NS - 2) * NPW) : "memory");
        __builtin_amdgcn_s_barrier();                  // (not __syncthreads: its fence waits vmcnt(0))
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kk = 0; kk < HK; ++kk) {
            if (kk < NPC)
#pragma unroll
                for (int p = kk * NPW / NPC; p < (kk + 1) * NPW / NPC; ++p) dma_piece(dst, t + NS, p);
            if (kk < RG) {
#pragma unroll
                for (int u = kk * UA / RG; u < (kk + 1) * UA / RG; ++u) OA::frag_unit(src, wm + c, h, u, ya);
#pragma unroll
                for (int u = kk * UB / RG; u < (kk + 1) * UB / RG; ++u) OB::frag_unit(src + IMG_A, wn + c, h, u, yb);
            }
            mfmas(kk, xa, xb);
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    float fa[MT][HK], fb[2][HK], ga[MT][HK], gb[2][HK];
#pragma unroll
    for (int i = 0; i < NS; ++i) dma(stg(i), i);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 1) * NPW) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int u = 0; u < UA; ++u) OA::frag_unit(s0, wm + c, h, u, fa);
#pragma unroll
    for (int u = 0; u < UB; ++u) OB::frag_unit(s0 + IMG_A, wn + c, h, u, fb);
    // step t + i of a trip (t a multiple of TRIP): its stage i % NS, the next one's (i + 1) % NS
    int t = 0;
    for (; t + TRIP <= nt; t += TRIP) {
#pragma unroll
        for (int i = 0; i < TRIP; i += 2) {
            step(t + i, stg(i % NS), stg((i + 1) % NS), fa, fb, ga, gb);
            step(t + i + 1, stg((i + 1) % NS), stg((i + 2) % NS), ga, gb, fa, fb);
        }
    }
    // the last nt - t < TRIP steps (a step's read of K-step nt and DMA past it are harmless); a
    // chain of exits, so no register set stays live across a join
#pragma unroll
    for (int i = 0; i < TRIP - 1; ++i) {
        if (t + i >= nt) break;
        if (i % 2 == 0) step(t + i, stg(i % NS), stg((i + 1) % NS), fa, fb, ga, gb);
        else step(t + i, stg(i % NS), stg((i + 1) % NS), ga, gb, fa, fb);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA outlives the workgroup

    // D map of the 32x32 forms: column = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    float* P = ws ? ws + (size_t)z * M * N : nullptr;
#pragma unroll
    for (int i = 0; i < MT; ++i)
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

// Direct-to-register form for the ~1k-token GEMMs (cfg 11): a 64×64 output tile per workgroup of
// 4 waves, each wave computing the whole 64×64 tile over every fourth K-step of the workgroup's K
// range (K-step t goes to wave t mod 4), with its operands loaded from global memory straight
// into the MFMA fragment registers: no LDS staging and no barrier in the K loop, and the next
// K-step's fragments in flight while this one's 64 MFMAs run.  The four partial tiles meet in
// LDS at the end and are summed in wave order (fixed: bitwise reproducible).  A 1.1k-token GEMM
// has 18 × 12..48 such tiles — one to four rounds over 256 CUs with every SIMD busy, where the
// 128×128 tile leaves 54 tiles for 256 CUs at N = 768 and needs a split-K workspace pass.
// Fragment registers of a lane (c = lane & 31, h = lane >> 5), K-step k0, MFMA step kk:
//   KC operand: row 32t + c of row tile t, k = k0 + 16h + kk — 64 contiguous bytes (4 × 16 B);
//   MC operand: rows 2c and 2c + 1, k = k0 + 16h + kk — one 8-B load per k-row; row tile t takes
//               row 2c + t (the permutation is undone where the partial tile goes to LDS).
template <bool KC>
struct SgDirect {
    static constexpr unsigned kOob = 0x7FFFFFF0u;     // past the descriptor's extent: loads return 0
    __amdgpu_buffer_rsrc_t rs;
    unsigned voff[2];
    int ld;

    __device__ void init(const float* src, int ld_, int rows, int row0, int lane) {
        ld = ld_;
        rs = sg_rsrc(src, kOob);
        const int c = lane & 31, h = lane >> 5;
        if (KC) {
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int r = row0 + 32 * t + c;
                voff[t] = r < rows ? (unsigned)((r * ld + 16 * h) * 4) : kOob;
            }
        } else {
            const int r = row0 + 2 * c;                   // rows % 4 == 0 (host-checked): r + 1 too
            voff[0] = r < rows ? (unsigned)((16 * h * ld + r) * 4) : kOob;
            voff[1] = 0;
        }
    }
    __device__ static int row(int t, int c) { return KC ? 32 * t + c : 2 * c + t; }
    // f[t][kk] = operand(row(t, c), k0 + 16h + kk).  TAIL: the K-step crosses ke, and k >= ke
    // reads as 0 (a select per load; only the last K-step of a split, outside the main loop).
    // (The loads' vectors are bit_cast whole: with their elements extracted one by one (v.x, v.y,
    // ...) hipcc / ROCm 7.2 shrank the 16-B load to ONE dword load — wrong values.)
    template <bool TAIL>
    __device__ __forceinline__ void load(float (&f)[2][16], int k0, int ke, int h) const {
        if (KC) {
            const int so = k0 * 4;
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    unsigned vo = voff[t] + 16 * q;
                    if (TAIL) vo = k0 + 16 * h + 4 * q < ke ? vo : kOob;
                    const float4 v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, so, 0));
                    f[t][4 * q] = v.x;
                    f[t][4 * q + 1] = v.y;
                    f[t][4 * q + 2] = v.z;
                    f[t][4 * q + 3] = v.w;
                }
        } else {
#pragma unroll
            for (int kk = 0; kk < 16; ++kk) {
                const int so = (k0 + kk) * ld * 4;
                unsigned vo = voff[0];
                if (TAIL) vo = k0 + 16 * h + kk < ke ? vo : kOob;
                const float2 v = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rs, vo, so, 0));
                f[0][kk] = v.x;
                f[1][kk] = v.y;
            }
        }
    }
};

constexpr int kD64Pitch = 72;                            // LDS row pitch (floats) of a partial tile
constexpr int kD64Smem = 4 * 64 * kD64Pitch * 4;         // 72 KiB: two workgroups per CU

template <bool AKC, bool BKC>
__global__ void __launch_bounds__(256, 2)
sgemm_d64_kernel(const float* __restrict__ A, int lda, const float* __restrict__ B, int ldb, float* __restrict__ C,
                 int ldc, int M, int N, int K, int kc, int accum, float* __restrict__ ws) {
    extern __shared__ __attribute__((aligned(16))) float part[];          // [wave][64 rows][kD64Pitch]
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int tm, tn, z;
    sg_tile((M + 63) / 64, (N + 63) / 64, tm, tn, z);
    const int m0 = tm * 64, n0 = tn * 64;
    const int kb = z * kc, ke = min(K, kb + kc);
    const int h = lane >> 5, c = lane & 31;
    SgDirect<AKC> oa;
    SgDirect<BKC> ob;
    oa.init(A, lda, M, m0, lane);
    ob.init(B, ldb, N, n0, lane);

    f32x16_t acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    auto mm = [&](const float (&xa)[2][16], const float (&xb)[2][16]) {
#pragma unroll
        for (int kk = 0; kk < 16; ++kk)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[i][kk], xb[j][kk], acc[i][j], 0, 0, 0);
    };
    // the workgroup's whole K-steps; this wave's: t = wave + 4 i, i < nw.  Every prefetch is
    // issued (a step past the wave's last re-reads its last one), so no load in the loop sits
    // under a branch — with conditional loads hipcc's waitcnt pass put vmcnt(0) before the MFMAs
    const int nt = (ke - kb) / 32, nw = nt > wave ? (nt - wave + 3) / 4 : 0;
    auto k_of = [&](int i) { return kb + 32 * (wave + 4 * min(i, nw - 1)); };
    float fa[2][16], fb[2][16], ga[2][16], gb[2][16];
    if (nw > 0) {
        oa.template load<false>(fa, k_of(0), ke, h);
        ob.template load<false>(fb, k_of(0), ke, h);
    }
    // two K-steps per trip, the register sets swapping roles: (f) = step i, (g) = step i + 1.
    // No branch inside a trip (hipcc sank a prefetch whose only use lay behind a branch down to
    // that use), sched_barriers keep each prefetch above the MFMAs that hide it; an odd last
    // step runs after the loop on (f), which the last trip's second prefetch filled.
    int i = 0;
    for (; i + 1 < nw; i += 2) {
        oa.template load<false>(ga, k_of(i + 1), ke, h);
        ob.template load<false>(gb, k_of(i + 1), ke, h);
        __builtin_amdgcn_sched_barrier(0);
        mm(fa, fb);
        __builtin_amdgcn_sched_barrier(0);
        oa.template load<false>(fa, k_of(i + 2), ke, h);
        ob.template load<false>(fb, k_of(i + 2), ke, h);
        __builtin_amdgcn_sched_barrier(0);
        mm(ga, gb);
        __builtin_amdgcn_sched_barrier(0);
    }
    if (i < nw) mm(fa, fb);
    // the partial K-step at the end of K (K % 32 != 0): the wave whose turn it is
    if (kb + 32 * nt < ke && wave == nt % 4) {
        oa.template load<true>(fa, kb + 32 * nt, ke, h);
        ob.template load<true>(fb, kb + 32 * nt, ke, h);
        mm(fa, fb);
    }

    // this wave's partial tile into LDS in (row, column) order
    // D map of the 32x32 forms: column = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    float* pw = part + wave * 64 * kD64Pitch;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                pw[SgDirect<AKC>::row(i, (r & 3) + 8 * (r >> 2) + 4 * h) * kD64Pitch + SgDirect<BKC>::row(j, c)] =
                    acc[i][j][r];
    __syncthreads();
    // wave w closes rows 16w .. 16w + 15: the four partials summed in wave order, 16 columns a lane
    const int ml = 16 * wave + (lane >> 2), cl = (lane & 3) * 16;
    const int row = m0 + ml;
    if (row >= M) return;
    float* P = ws ? ws + (size_t)z * M * N : nullptr;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int col = n0 + cl + 4 * q;
        if (col >= N) break;                              // N % 4 == 0: whole float4s
        const int o = ml * kD64Pitch + cl + 4 * q;
        float4 s = *(const float4*)(part + o);
#pragma unroll
        for (int p = 1; p < 4; ++p) {
            const float4 v = *(const float4*)(part + p * 64 * kD64Pitch + o);
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
        if (P) {
            *(float4*)(P + (size_t)row * N + col) = s;
        } else {
            float4* d = (float4*)(C + (size_t)row * ldc + col);
            if (accum) {
                const float4 v = *d;
                s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
            }
            *d = s;
        }
    }
}

// Stream-K form of the 128×128 kernel (the default): a persistent grid of G workgroups (two
// per CU) first takes dp whole tiles each (round r: tile r·G + d), then splits the remaining
// tiles' K-steps evenly — workgroup d takes iterations [d·I/G, (d+1)·I/G) of the flattened
// (tile, K-step) space, so every CU ends with the same number of K-steps instead of a half-empty
// last round or a split-K workspace pass.  A workgroup's first segment that starts inside a tile
// is a partial: stored to ws[d] (sc1 write-through 16-B stores, every wave drained, then one
// lane's sc1 flag store of this launch's epoch — MI355X_MICROARCH inter-workgroup visibility,
// table row 1); the tile's owner (the workgroup holding its first K-step) polls the flags of the
// workgroups after it and adds their partials (sc1 loads) in K order, so the sum order is fixed
// by (shape, G) alone and a step stays bitwise reproducible.  Partials come first in every
// workgroup's stream and owners wait only on later workgroups, so no wait chains; the grid fits
// the chip at two per CU (every workgroup resident), and the poll is bounded (a timeout sets
// flags[kSkTimeout]; the trainer step fails).
constexpr int kSkMaxG = 512, kSkTimeout = 1023;    // flag words: [0, G) epochs, [1023] timeout

template <bool AKC, bool BKC>
__global__ void __launch_bounds__(256, 2)
sgemm_sk_kernel(const float* __restrict__ A, int lda, const float* __restrict__ B, int ldb, float* __restrict__ C,
                int ldc, int M, int N, int K, int accum, float* __restrict__ ws, unsigned* __restrict__ flags,
                unsigned epoch, int dp, long long sk_iters, int sk_tile0) {
    constexpr int BM = 128, BN = 128, TM = 64, BK = 32;
    constexpr int WM = BM / TM, NW = 4, MT = TM / 32, HK = BK / 2;
    constexpr int IMG_A = BM * BK * 4, STAGE = (BM + BN) * BK * 4;
    using OA = SgOperand<AKC, BM, NW, BK>;
    using OB = SgOperand<BKC, BN, NW, BK>;
    typedef __attribute__((address_space(1))) unsigned gu32;
    typedef int i4 __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int G = gridDim.x;
    // XCD-contiguous workgroup index (blocks b and b + 8 share an XCD): neighbours d, d + 1 —
    // a partial's producer and its owner — mostly share an L2
    int d;
    {
        const int b = blockIdx.x, xcd = b & 7, pos = b >> 3, q = G >> 3, r = G & 7;
        d = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
    }
    const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
    const int steps = (K + BK - 1) / BK;
    auto tile_rc = [&](int u, int& m0, int& n0) {            // groups of 8 row panels, column-walked
        constexpr int GM = 8;
        const int g = u / (GM * tiles_n), loc = u - g * GM * tiles_n;
        const int gm = min(GM, tiles_m - g * GM);
        const int tn = loc / gm;
        m0 = (g * GM + (loc - tn * gm)) * BM;
        n0 = tn * BN;
    };
    const int wm = (wave % WM) * TM, wn = (wave / WM) * 64;
    const int h = lane >> 5, c = lane & 31;
    const __amdgpu_buffer_rsrc_t wrs = sg_rsrc(ws, 0x7FFFFFF0u);
    f32x16_t acc[MT][2];

    // K-steps [s0, s1) of the tile at (m0, n0) into acc (zeroed first)
    auto run = [&](int m0, int n0, int s0, int s1) {
        OA oa;
        OB ob;
        oa.init(A, lda, M, m0, wave, lane);
        ob.init(B, ldb, N, n0, wave, lane);
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
        __syncthreads();                               // every wave done with the previous tile's LDS
        oa.stage(smem, wave, s0 * BK, K);
        ob.stage(smem + IMG_A, wave, s0 * BK, K);
        int buf = 0;
        for (int st = s0; st < s1; ++st) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            const char* sb = smem + buf * STAGE;
            float fa[MT][HK], fb[2][HK];
#pragma unroll
            for (int i = 0; i < MT; ++i) OA::frag(sb, wm + 32 * i + c, h, fa[i]);
#pragma unroll
            for (int j = 0; j < 2; ++j) OB::frag(sb + IMG_A, wn + 32 * j + c, h, fb[j]);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            if (st + 1 < s1) {
                char* nx = smem + (buf ^ 1) * STAGE;
                oa.stage(nx, wave, (st + 1) * BK, K);
                ob.stage(nx + IMG_A, wave, (st + 1) * BK, K);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int kk = 0; kk < HK; ++kk)
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][kk], fb[j][kk], acc[i][j], 0, 0, 0);
            buf ^= 1;
        }
    };
    // D map of the 32x32 forms: column = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    auto store_c = [&](int m0, int n0) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int col = n0 + wn + 32 * j + c;
                if (col >= N) continue;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
                    if (row >= M) continue;
                    float* o = C + (size_t)row * ldc + col;
                    *o = accum ? acc[i][j][r] + *o : acc[i][j][r];
                }
            }
    };
    // partial slot of workgroup w: [wave][i][j][lane][16] floats, 16-B pieces
    auto part_off = [&](int w, int i, int j, int q) {
        return (int)((((size_t)w * 16384 + wave * 4096 + ((i * 2 + j) * 64 + lane) * 16) + 4 * q) * 4);
    };

    for (int rr = 0; rr < dp; ++rr) {                  // data-parallel rounds: whole tiles
        int m0, n0;
        tile_rc(rr * G + d, m0, n0);
        run(m0, n0, 0, steps);
        store_c(m0, n0);
    }
    const long long b0 = (long long)d * sk_iters / G, b1 = (long long)(d + 1) * sk_iters / G;
    for (long long it = b0; it < b1;) {
        const int u = sk_tile0 + (int)(it / steps);
        const int s0 = (int)(it % steps);
        const long long tile_end = (long long)(u - sk_tile0 + 1) * steps;
        const int s1 = (int)(min(tile_end, b1) - (long long)(u - sk_tile0) * steps);
        int m0, n0;
        tile_rc(u, m0, n0);
        run(m0, n0, s0, s1);
        if (s0 > 0) {
            // a partial (this workgroup's first segment): publish it to the tile's owner
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const f32x4 v = {acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
                        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i4, v), wrs, part_off(d, i, j, q), 0, 16);
                    }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");          // every storing wave drains
            __syncthreads();
            if (tid == 0) __hip_atomic_store((gu32*)(flags + d), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            // the owner: the partials of the workgroups after it, in K order
            long long cov = (long long)(u - sk_tile0) * steps + s1;     // covered up to (flat)
            for (int w = d + 1; cov < tile_end && w < G; ++w) {
                const long long wb0 = (long long)w * sk_iters / G, wb1 = (long long)(w + 1) * sk_iters / G;
                if (wb0 == wb1) continue;                  // an empty range publishes nothing
                if (tid == 0) {
                    for (unsigned spins = 0; __hip_atomic_load((gu32*)(flags + w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch;) {
                        __builtin_amdgcn_s_sleep(2);
                        if (++spins == (1u << 22)) {
                            __hip_atomic_store((gu32*)(flags + kSkTimeout), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            break;
                        }
                    }
                }
                __syncthreads();
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(wrs, part_off(w, i, j, q), 0, 16));
                            acc[i][j][4 * q] += v[0];
                            acc[i][j][4 * q + 1] += v[1];
                            acc[i][j][4 * q + 2] += v[2];
                            acc[i][j][4 * q + 3] += v[3];
                        }
                cov = min(tile_end, wb1);
            }
            store_c(m0, n0);
        }
        it = min(tile_end, b1);
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

// Tile configurations (RS_SGEMM_CFG indices; the retired ones — measured, never picked, their
// instantiations removed — keep their index and fail with hipErrorInvalidValue):
//   0  128×128×32 sgemm_dma_kernel, 4 waves of 64×64, 2 workgroups per CU (the round-3 default)
//   9  192×128×32 sgemm_dma_kernel, 4 waves of 96×64
//   11 64×64 sgemm_d64_kernel (direct to registers)
//   12 128×128 sgemm_sp_kernel (software-pipelined; the round-6 default), 17 / 18 its 64×128 /
//      128×64 half tiles (4 waves of 32×64)
//   retired: 1-8 and 10 (sgemm_dma_kernel at BK 16, 128×64, 64×64, 256×128, 256×256; the round-2
//   3-stage sgemm_pipe_kernel; profiles/r5e_sgemm_all.jsonl), 13-16 and 19 (sgemm_sp_kernel at
//   3 / 4 stages, 192×128, 256×128, 64×64; profiles/r6y_sgemm_split_sweep.txt, r6aa_*)
struct SgCfg { int bm, bn, bk, occ, live; };
constexpr int kSgNCfg = 20;
constexpr SgCfg kSgCfg[kSgNCfg] = {{128, 128, 32, 2, 1}, {128, 128, 16, 4, 0}, {256, 128, 32, 1, 0},
                                   {128, 128, 16, 3, 0}, {128, 128, 32, 1, 0}, {128, 64, 32, 2, 0},
                                   {128, 64, 32, 3, 0},  {64, 64, 32, 4, 0},   {64, 64, 32, 6, 0},
                                   {192, 128, 32, 2, 1}, {256, 256, 32, 1, 0}, {64, 64, 32, 2, 1},
                                   {128, 128, 32, 2, 1}, {192, 128, 32, 1, 0}, {256, 128, 32, 1, 0},
                                   {128, 128, 32, 1, 0}, {128, 128, 32, 1, 0}, {64, 128, 32, 2, 1},
                                   {128, 64, 32, 2, 1},  {64, 64, 32, 4, 0}};

// Modelled time (µs) of one configuration at a split count: dispatch rounds × (K-steps per
// workgroup × the time a CU takes per K-step with its resident workgroups + a per-round
// prologue/epilogue), plus, split, the partials' round trip.  Fitted to the forced-split sweep of
// the 128×128 tile (profiles/r3_sgemm_split_sweep.txt, 135 points, 5 % rms): 3.74 µs per K-step
// with two workgroups on the CU, 2.14 alone (a grid of at most one workgroup per CU is spread
// one per CU; a partial last round of a larger grid is packed two per CU and costs a whole
// round), 5.4 µs per round, 4.2 µs + (2·splits + 1)·M·N·4 B at 7.9 TB/s for the partials; the
// weight-gradient form (both operands output-contiguous, ds_read_b32 fragments) 10 % slower per
// step.  192×128: 6.4 / 3.4 µs per K-step (profiles/r3u_sgemm_pick.txt).  Other tiles scale by
// their K-step volume.
int n_cus_sg();

// `cus`: the device's CU count (n_cus_sg() on the trainer's path; an explicit value in the host-only
// picker test), so the pick is a function of the shape and the CU count
double sg_model(int cfg, int M, int N, int K, int sp, bool mcmc, int cus_) {
    const SgCfg& g = kSgCfg[cfg];
    const long long tiles = (long long)((M + g.bm - 1) / g.bm) * ((N + g.bn - 1) / g.bn);
    const int steps = (K + g.bk - 1) / g.bk, per = (steps + sp - 1) / sp, spr = (steps + per - 1) / per;
    const double vol = (double)g.bm * g.bn * g.bk / (128.0 * 128.0 * 32.0);
    double t_one = 2.14 * vol, t_full = 3.74 * vol * g.occ / 2.0;
    const long long wgs = tiles * spr, cus = cus_;
    double t;
    if (cfg >= 12) {
        // software-pipelined tiles: a CU retires a workgroup's K-step in the same time alone as
        // beside a second one (the LDS reads and the barrier no longer idle the MFMA pipe), so
        // the time is the K-steps of the most loaded CU, ceil(wgs / CUs) workgroups.  Fitted to
        // the split sweep of the 27 training shapes (profiles/r6y_sgemm_split_sweep.txt, 135
        // points, 3.4 % rms): 1.745 µs per 128×128 K-step, 1.94 µs per workgroup, 8.0 µs, and for
        // a split 0.52 µs + 0.121 µs per MB of partials written and read
        // (per workgroup 0.66 + 1.28 vol, fixed 5.4 + 2.6 vol: the 64×128 / 128×64 tiles' 1.27 and
        // 6.7 fitted to their 1100-token sweep, profiles/r6aa_sgemm_small_tiles.txt, 2.9 % rms)
        const long long rounds = (wgs + cus - 1) / cus;
        t = 1.745 * vol * rounds * per + (0.66 + 1.28 * vol) * rounds + 5.4 + 2.6 * vol;
        if (spr > 1) t += 0.52 + 0.121e-6 * (2.0 * spr + 1.0) * M * N * 4.0;
        return t;
    }
    if (cfg == 11) {
        // 64×64 direct-to-register tiles: a wave runs every fourth K-step.  One pass (at most one
        // workgroup per CU): 2.1 µs per wave K-step + 8 µs (profiles/r6y_sgemm_split_sweep.txt,
        // split 1, 8 shapes, 0.85-1.2x); otherwise small workgroups are dispatched as slots free
        // up, so the load is continuous in the grid size rather than in whole rounds, fitted to
        // the 27 training shapes (profiles/r4f_sgemm_cfg11.txt, 9 % rms): 1.55 µs per wave K-step
        // alone, 4.5 µs per K-step-round at two workgroups per CU, 10 µs
        if (wgs <= cus) return 8.0 + 2.1 * ((per + 3) / 4) + (spr > 1 ? 4.24 + (2.0 * spr + 1.0) * M * N * 4.0 * 0.127e-6 : 0.0);
        t = 10.0 + (per + 3) / 4 * std::max(1.55, (double)wgs / (cus * g.occ) * 4.5);
    } else {
        if (cfg == 9) { t_one = 3.43; t_full = 6.4; }
        else if (mcmc) { t_one *= 1.1; t_full *= 1.1; }
        t = wgs <= cus ? per * t_one + 5.44
                       : (double)((wgs + cus * g.occ - 1) / (cus * g.occ)) * (per * t_full + 5.44);
    }
    if (spr > 1) t += 4.24 + (2.0 * spr + 1.0) * M * N * 4.0 * 0.127e-6;
    return t;
}

int sg_splits(int cfg, int M, int N, int K, int* kc, bool mcmc, int cus) {
    const SgCfg& g = kSgCfg[cfg];
    const int steps = (K + g.bk - 1) / g.bk;
    // the split count with the lowest modelled time (at least 4 K-steps per split).
    // RS_SGEMM_SPLITS forces a split count (A/B knob).
    static const int forced = [] {
        const char* v = getenv("RS_SGEMM_SPLITS");
        return v ? std::max(1, atoi(v)) : 0;
    }();
    int splits = 1;
    if (forced) {
        splits = std::min(forced, std::max(1, steps));
    } else {
        double best = 1e30;
        const long long tiles = (long long)((M + g.bm - 1) / g.bm) * ((N + g.bn - 1) / g.bn);
        for (int sp = 1; sp <= 16 && sp <= std::max(1, steps / 4); ++sp) {
            // software-pipelined tiles: no split past two workgroups per CU (a third round of
            // short splits measured well above the model: profiles/r6y_sgemm_split_sweep.txt)
            const int per_ = (steps + sp - 1) / sp;
            if (cfg >= 12 && sp > 1 && tiles * ((steps + per_ - 1) / per_) > 2LL * cus) break;
            const double t = sg_model(cfg, M, N, K, sp, mcmc, cus);
            if (t < best) {
                best = t;
                splits = sp;
            }
        }
    }
    const int per = (steps + splits - 1) / splits;
    *kc = per * g.bk;
    return (steps + per - 1) / per;
}

// The tile configuration: the software-pipelined 128×128 tile (cfg 12) at its best split, a
// software-pipelined 64×128 / 128×64 tile (cfg 17 / 18) where it wins by 3 % (the ~1k-token
// GEMMs: twice the tiles for the same rounds), or the 64×64 direct-to-register form (cfg 11)
// where its grid is one pass and it times lower (1100 × 768 × 768: 216 tiles).  Against rocBLAS / hipBLASLt at the 27 training shapes: profiles/r6*_sgemm_all.jsonl.
// RS_SGEMM_CFG forces a live configuration (A/B knob).  The choice depends on the shape and the
// device's CU count only, so a shape's results stay bitwise reproducible on a given device model.
int sg_pick(int M, int N, int K, bool mcmc, int cus) {
    static const int forced = [] {
        const char* v = getenv("RS_SGEMM_CFG");
        return v ? atoi(v) : -1;
    }();
    if (forced >= 0 && forced < kSgNCfg && kSgCfg[forced].live) return forced;
    int kc = 0, best = 12;
    double tb = sg_model(12, M, N, K, sg_splits(12, M, N, K, &kc, mcmc, cus), mcmc, cus);
    for (int cfg : {17, 18}) {                    // a half tile where it wins by 3 %
        const double t = sg_model(cfg, M, N, K, sg_splits(cfg, M, N, K, &kc, mcmc, cus), mcmc, cus);
        if (t < 0.97 * tb) {
            tb = t;
            best = cfg;
        }
    }
    // the 64×64 direct form where its grid is one pass (no split) and it times lower
    const long long tiles64 = (long long)((M + 63) / 64) * ((N + 63) / 64);
    return tiles64 <= cus && sg_model(11, M, N, K, 1, mcmc, cus) < tb ? 11 : best;
}

bool sk_enabled() {                                 // read per call (tests flip it in-process)
    const char* e = getenv("RS_SGEMM_SK");
    return e && !strcmp(e, "1");
}

int n_cus_sg() {
    static int n = [] {
        int dev = 0, v = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
        return v > 0 ? v : 256;
    }();
    return n;
}

// Stream-K hand-off words of the current device: 1024 zeroed words (epoch tags [0, 512), the
// timeout word), allocated on first use; the epoch counts launches (never 0, so a zeroed or
// stale word never matches).  Single-threaded use, as the trainer's.
struct SkFlags {
    unsigned* p = nullptr;
    unsigned epoch = 0;
};
SkFlags g_sk[16];

hipError_t sk_flags(unsigned** f, unsigned* epoch) {
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev)) return e;
    SkFlags& k = g_sk[dev & 15];
    if (!k.p) {
        if (hipError_t e = hipMalloc((void**)&k.p, 1024 * 4)) return e;
        if (hipError_t e = hipMemset(k.p, 0, 1024 * 4)) return e;
    }
    if (++k.epoch == 0) k.epoch = 1;
    *f = k.p;
    *epoch = k.epoch;
    return hipSuccess;
}

}  // namespace

// 1 when a stream-K owner gave up waiting for a partial since the last call (cleared by it)
int tr_sgemm_failed() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    SkFlags& k = g_sk[dev & 15];
    if (!k.p) return 0;
    unsigned v = 0;
    if (hipMemcpy(&v, k.p + kSkTimeout, 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    if (v) (void)hipMemset(k.p + kSkTimeout, 0, 4);
    return v != 0;
}

size_t tr_sgemm_ws_floats(int M, int N, int K) {
    size_t w = sk_enabled() ? (size_t)kSkMaxG * 16384 : 0;   // stream-K partial slots (128×128 each)
    for (int cfg = 0; cfg < kSgNCfg; ++cfg) {  // any configuration the picker or the knob may choose
        if (!kSgCfg[cfg].live) continue;
        int kc = 0;
        for (int mc = 0; mc < 2; ++mc) {
            const int s = sg_splits(cfg, M, N, K, &kc, mc != 0, n_cus_sg());
            if (s > 1) w = std::max(w, (size_t)s * M * N);
        }
    }
    return w;
}

static hipError_t sg_run(int cfg, int M, int N, int K, const float* A, int lda, bool a_kc, const float* B, int ldb,
                         bool b_kc, float* C, int ldc, int accum, float* ws, size_t ws_floats, hipStream_t s) {
    if (M <= 0 || N <= 0) return hipSuccess;
    // 16-B DMA pieces along each operand's contiguous dimension, float4 rows of C (split-K sum)
    if (N % 4 || lda % 4 || ldb % 4 || ldc % 4 || (a_kc ? K % 4 : M % 4) || (b_kc ? K % 4 : N % 4) ||
        ((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) % 16 || cfg < 0 || cfg >= kSgNCfg || !kSgCfg[cfg].live)
        return hipErrorInvalidValue;
    // 32-bit byte offsets into each operand (buffer descriptors)
    const long long ea = (long long)(a_kc ? M : K) * lda * 4, eb = (long long)(b_kc ? N : K) * ldb * 4;
    if (ea >= 0x7FFFFFF0ll || eb >= 0x7FFFFFF0ll) return hipErrorInvalidValue;
    if (K <= 0) {   // empty reduction: C = 0 (+ C)
        if (accum) return hipSuccess;
        for (int r = 0; r < M; ++r) {
            hipError_t e = hipMemsetAsync(C + (size_t)r * ldc, 0, (size_t)N * 4, s);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    // cfg 0 with RS_SGEMM_SK=1: the stream-K kernel instead of the split-K form (opt-in: its
    // owner-side fix-up — poll, then 64 KB per partial read by one workgroup — cost more than
    // the chip-wide workspace sum on all but one training shape, profiles/r3_sgemm_streamk.txt)
    if (cfg == 0 && sk_enabled()) {
        const int tiles = ((M + 127) / 128) * ((N + 127) / 128), steps = (K + 31) / 32;
        const int G = std::min(std::min(kSkMaxG, 2 * n_cus_sg()), tiles * steps);
        if (!ws || ws_floats < (size_t)G * 16384) return hipErrorInvalidValue;
        unsigned* flags = nullptr;
        unsigned epoch = 0;
        if (hipError_t e = sk_flags(&flags, &epoch)) return e;
        int dp = tiles / G;
        const int rem = tiles - dp * G;
        if (rem * 10 >= G * 9) ++dp;               // a nearly full last round: whole tiles, no partials
        const int sk_tile0 = std::min(tiles, dp * G);
        const long long sk_iters = (long long)(tiles - sk_tile0) * steps;
#define SK_LAUNCH(AK, BK_)                                                                                      \
    hipLaunchKernelGGL((sgemm_sk_kernel<AK, BK_>), dim3(G), dim3(256), 0, s, A, lda, B, ldb, C, ldc, M, N, K, accum, \
                       ws, flags, epoch, dp, sk_iters, sk_tile0)
        if (a_kc && b_kc) SK_LAUNCH(true, true);
        else if (a_kc) SK_LAUNCH(true, false);
        else if (b_kc) SK_LAUNCH(false, true);
        else SK_LAUNCH(false, false);
#undef SK_LAUNCH
        return hipGetLastError();
    }
    int kc = 0;
    const int splits = sg_splits(cfg, M, N, K, &kc, !a_kc && !b_kc, n_cus_sg());
    float* P = nullptr;
    if (splits > 1) {
        if (!ws || ws_floats < (size_t)splits * M * N) return hipErrorInvalidValue;
        P = ws;
    }
    const SgCfg& g = kSgCfg[cfg];
    const dim3 grid(((N + g.bn - 1) / g.bn) * ((M + g.bm - 1) / g.bm) * splits);   // sg_tile remaps
#define SG_LAUNCH(KER, AK, BK_, BM_, BN_, TM_, KB_, OCC_)                                                    \
    hipLaunchKernelGGL((KER<AK, BK_, BM_, BN_, TM_, KB_, OCC_>), grid, dim3((BM_ / TM_) * (BN_ / 64) * 64), 0, s, \
                       A, lda, B, ldb, C, ldc, M, N, K, kc, accum, P)
#define SG_FORMS(KER, BM_, BN_, TM_, KB_, OCC_)                                   \
    do {                                                                          \
        if (a_kc && b_kc) SG_LAUNCH(KER, true, true, BM_, BN_, TM_, KB_, OCC_);   \
        else if (a_kc) SG_LAUNCH(KER, true, false, BM_, BN_, TM_, KB_, OCC_);     \
        else if (b_kc) SG_LAUNCH(KER, false, true, BM_, BN_, TM_, KB_, OCC_);     \
        else SG_LAUNCH(KER, false, false, BM_, BN_, TM_, KB_, OCC_);              \
    } while (0)
#define SP_LAUNCH(AK, BK_, BM_, BN_, TM_, NS_, OCC_)                                                          \
    hipLaunchKernelGGL((sgemm_sp_kernel<AK, BK_, BM_, BN_, TM_, NS_, OCC_>), grid, dim3((BM_ / TM_) * (BN_ / 64) * 64), \
                       0, s, A, lda, B, ldb, C, ldc, M, N, K, kc, accum, P)
#define SP_FORMS(BM_, BN_, TM_, NS_, OCC_)                                     \
    do {                                                                       \
        if (a_kc && b_kc) SP_LAUNCH(true, true, BM_, BN_, TM_, NS_, OCC_);     \
        else if (a_kc) SP_LAUNCH(true, false, BM_, BN_, TM_, NS_, OCC_);       \
        else if (b_kc) SP_LAUNCH(false, true, BM_, BN_, TM_, NS_, OCC_);       \
        else SP_LAUNCH(false, false, BM_, BN_, TM_, NS_, OCC_);                \
    } while (0)
    if (cfg == 0) SG_FORMS(sgemm_dma_kernel, 128, 128, 64, 32, 2);
    else if (cfg == 9) SG_FORMS(sgemm_dma_kernel, 192, 128, 96, 32, 2);
    else if (cfg == 12) SP_FORMS(128, 128, 64, 2, 2);
    else if (cfg == 17) SP_FORMS(64, 128, 32, 2, 2);
    else if (cfg == 18) SP_FORMS(128, 64, 32, 2, 2);
    else {
        static const hipError_t attr = [] {
            for (const void* f : {(const void*)sgemm_d64_kernel<true, true>, (const void*)sgemm_d64_kernel<true, false>,
                                  (const void*)sgemm_d64_kernel<false, true>, (const void*)sgemm_d64_kernel<false, false>})
                if (hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kD64Smem)) return e;
            return hipSuccess;
        }();
        if (attr != hipSuccess) return attr;
#define D64_LAUNCH(AK, BK_)                                                                                    \
    hipLaunchKernelGGL((sgemm_d64_kernel<AK, BK_>), grid, dim3(256), kD64Smem, s, A, lda, B, ldb, C, ldc, M, N, K, kc, \
                       accum, P)
        if (a_kc && b_kc) D64_LAUNCH(true, true);
        else if (a_kc) D64_LAUNCH(true, false);
        else if (b_kc) D64_LAUNCH(false, true);
        else D64_LAUNCH(false, false);
#undef D64_LAUNCH
    }
#undef SP_FORMS
#undef SP_LAUNCH
#undef SG_FORMS
#undef SG_LAUNCH
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || splits == 1) return e;
    const size_t n4 = (size_t)M * N / 4;
    hipLaunchKernelGGL(sgemm_splitk_sum_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, P, splits, M, N, C,
                       ldc, accum);
    return hipGetLastError();
}

hipError_t tr_sgemm(int M, int N, int K, const float* A, int lda, bool a_kc, const float* B, int ldb, bool b_kc,
                    float* C, int ldc, int accum, float* ws, size_t ws_floats, hipStream_t s) {
    return sg_run(sg_pick(M, N, K, !a_kc && !b_kc, n_cus_sg()), M, N, K, A, lda, a_kc, B, ldb, b_kc, C, ldc, accum, ws, ws_floats, s);
}

// Test / timing entry (not part of the scoring path): one trainer GEMM in the given operand
// form (cfg -1: the shape's pick, 0..2: a tile configuration); the split-K workspace is a
// grow-only buffer kept across calls (single-threaded use).  Returns 0 on success.
extern "C" int rs_debug_sgemm_cfg(int cfg, int M, int N, int K, const float* A, int lda, int a_kc, const float* B,
                                  int ldb, int b_kc, float* C, int ldc, int accum, void* stream) {
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
    hipError_t e = sg_run(cfg < 0 ? sg_pick(M, N, K, a_kc == 0 && b_kc == 0, n_cus_sg()) : cfg, M, N, K, A, lda, a_kc != 0, B, ldb, b_kc != 0, C, ldc,
                          accum, ws, ws_cap, (hipStream_t)stream);
    return e == hipSuccess ? 0 : -2;
}

extern "C" int rs_debug_sgemm(int M, int N, int K, const float* A, int lda, int a_kc, const float* B, int ldb, int b_kc,
                              float* C, int ldc, int accum, void* stream) {
    return rs_debug_sgemm_cfg(-1, M, N, K, A, lda, a_kc, B, ldb, b_kc, C, ldc, accum, stream);
}

// Test entry (host only, no GPU call): the tile configuration and split count the trainer's
// picker chooses for a GEMM shape on a device of `cus` CUs (100 · cfg + splits; mcmc = both
// operands output-contiguous, the weight-gradient form).
extern "C" int rs_debug_sgemm_pick(int M, int N, int K, int mcmc, int cus) {
    if (cus <= 0) return -1;
    const int cfg = sg_pick(M, N, K, mcmc != 0, cus);
    int kc = 0;
    const int sp = sg_splits(cfg, M, N, K, &kc, mcmc != 0, cus);
    return 100 * cfg + sp;
}
