// BERT encoder kernels other than the GEMMs (gfx950, wave64).
//
//  embed_ln        K1+K2: on-device [MASK] expansion (MLM_PLL/preprocess.py:15-21) fused with
//                  BertEmbeddings (modeling_bert.py:53-108): word + type[0] + position -> LN
//  ln_rows         LayerNorm of BertSelfOutput / BertOutput / head transform (eps 1e-12)
//  attention_full  eager_attention_forward (modeling_bert.py:111-136) over ragged sequences
//                  (no padding rows: equal to the reference's additive pad mask)
//  attention_query the same, last layer, only the scored row of each sequence (masked
//                  position for MLM_PLL, [CLS] for RescoreBert) — the other rows' last-layer
//                  states never reach a score
//  lse_finalize    merges the decoder epilogue's (max, sum exp) slabs: log_softmax gather
//                  (MLM_PLL/main.py:101-105)
//  cls_linear      RescoreBert Linear(H, 1) on the CLS state (RescoreBert/model.py:19-20)
//  segsum_f64      per-hypothesis PLL, float64, in row order (MLM_PLL/main.py:106-107)
//
// Every producer of a GEMM operand writes the fp16 operand image (put_split: [hi],
// [hi | hi/64 | lo*64], or the split-operand form's per-K-step interleaved [hi 32 | lo 32]).  The residual stream stays PRE-LayerNorm in fp32 (x32) with per-row
// (mean, rstd): its consumers (the next residual GEMM's accumulator init, attention_query)
// rebuild LN(x) with ln_apply, so no LN kernel writes an fp32 copy of its output.
#include <type_traits>
#include "common.h"
#include <stdlib.h>
#include <string.h>

namespace {

// LayerNorm of one row held as NV float4 per lane (row = 256*NV floats over one wave).
// Writes the row statistics (stats != null), LN(x) in fp32 (y32 != null) and the fp16
// operand image; every output element goes through ln_apply (common.h).
template <int NV>
__device__ __forceinline__ void ln_store(const float4 (&x)[NV], const float* g, const float* b, float eps,
                                         int lane, float* y32, float2* stats, f16* y16, int kx) {
    constexpr int H = NV * 256;
    float s = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v) s += (x[v].x + x[v].y) + (x[v].z + x[v].w);
    const float mean = __fmul_rn(wave_sum(s), 1.0f / H);
    float q = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const float4 d = make_float4(x[v].x - mean, x[v].y - mean, x[v].z - mean, x[v].w - mean);
        q += __builtin_fmaf(d.x, d.x, __fmul_rn(d.y, d.y)) + __builtin_fmaf(d.z, d.z, __fmul_rn(d.w, d.w));
    }
    const float2 st = make_float2(mean, 1.0f / sqrtf(__builtin_fmaf(wave_sum(q), 1.0f / H, eps)));
    if (stats && lane == 0) *stats = st;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int c = v * 256 + lane * 4;
        const float4 gg = *(const float4*)(g + c);
        const float4 bb = *(const float4*)(b + c);
        float4 y;
        y.x = ln_apply(x[v].x, st, gg.x, bb.x);
        y.y = ln_apply(x[v].y, st, gg.y, bb.y);
        y.z = ln_apply(x[v].z, st, gg.z, bb.z);
        y.w = ln_apply(x[v].w, st, gg.w, bb.w);
        if (y32) *(float4*)(y32 + c) = y;
        if (y16) put_split4(y16, c, H, kx, y);
    }
}

// Embedding sum of position t of a sequence (token t, or [MASK] when t == mp): the one
// expression both the copy-row and the unique-row kernels use (bit-identical rows).
template <int NV>
__device__ __forceinline__ void embed_row(const int* tok, int toff, int t, int mp, int mask_id, int vocab,
                                          const float* word, const float* pos, const float* type0, int lane,
                                          float4 (&x)[NV]) {
    constexpr int H = NV * 256;
    int id = (t == mp) ? mask_id : tok[toff + t];
    id = min(max(id, 0), vocab - 1);              // out-of-range ids are clamped, never read OOB
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int c = v * 256 + lane * 4;
        const float4 w = *(const float4*)(word + (size_t)id * H + c);
        const float4 ty = *(const float4*)(type0 + c);
        const float4 p = *(const float4*)(pos + (size_t)t * H + c);
        // transformers order: (inputs_embeds + token_type) + position
        x[v] = make_float4((w.x + ty.x) + p.x, (w.y + ty.y) + p.y, (w.z + ty.z) + p.z, (w.w + ty.w) + p.w);
    }
}

// Layer-0 dedup: block s writes the [MASK] unique row of sequence s, and — when s is the
// first copy of its hypothesis in the chunk — the hypothesis' T unmasked unique rows.
template <int NV>
__global__ void __launch_bounds__(256)
embed_unique_kernel(const int* __restrict__ tok, SeqMeta sm, int s0, int mask_id, int vocab,
                    const float* __restrict__ word, const float* __restrict__ pos,
                    const float* __restrict__ type0, const float* __restrict__ g,
                    const float* __restrict__ b, float eps, f16* __restrict__ h16u, int kx) {
    constexpr int H = NV * 256;
    const int s = s0 + blockIdx.x;
    const int T = sm.len[s], toff = sm.tok_off[s], mp = sm.mask_pos[s];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const bool first = blockIdx.x == 0 || sm.urow_h[s - 1] != sm.urow_h[s];
    const int n = first ? T + 1 : 1;
    for (int k = wave; k < n; k += 4) {
        const bool masked = k == T || !first;
        const int t = masked ? mp : k;
        const size_t r = masked ? (size_t)sm.urow_m[s] : (size_t)(sm.urow_h[s] + k);
        float4 x[NV];
        embed_row<NV>(tok, toff, t, masked ? t : -1, mask_id, vocab, word, pos, type0, lane, x);
        ln_store<NV>(x, g, b, eps, lane, nullptr, nullptr, h16u + r * kx * H, kx);
    }
}

template <int NV>
__global__ void __launch_bounds__(256)
embed_ln_kernel(const int* __restrict__ tok, SeqMeta sm, int s0, int row0, int mask_id, int vocab,
                const float* __restrict__ word, const float* __restrict__ pos,
                const float* __restrict__ type0, const float* __restrict__ g,
                const float* __restrict__ b, float eps, float* __restrict__ x32,
                float2* __restrict__ stats, f16* __restrict__ h16, int kx) {
    constexpr int H = NV * 256;
    const int s = s0 + blockIdx.x;
    const int T = sm.len[s], toff = sm.tok_off[s], mp = sm.mask_pos[s];
    const int rs = sm.row[s] - row0;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int t = wave; t < T; t += 4) {
        float4 x[NV];
        embed_row<NV>(tok, toff, t, mp, mask_id, vocab, word, pos, type0, lane, x);
        const size_t r = (size_t)(rs + t);
#pragma unroll
        for (int v = 0; v < NV; ++v) if (x32) *(float4*)(x32 + r * H + v * 256 + lane * 4) = x[v];
        ln_store<NV>(x, g, b, eps, lane, nullptr, stats ? stats + r : nullptr, h16 ? h16 + r * kx * H : nullptr, kx);
    }
}

template <int NV>
__global__ void __launch_bounds__(256)
ln_rows_kernel(const float* __restrict__ xin, int rows, const float* __restrict__ g,
               const float* __restrict__ b, float eps, float* __restrict__ y32,
               float2* __restrict__ stats, f16* __restrict__ y16, int kx) {
    constexpr int H = NV * 256;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    float4 x[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) x[v] = *(const float4*)(xin + (size_t)row * H + v * 256 + lane * 4);
    ln_store<NV>(x, g, b, eps, lane, y32 ? y32 + (size_t)row * H : nullptr, stats ? stats + row : nullptr,
                 y16 + (size_t)row * kx * H, kx);
}

// BertSelfOutput (modeling_bert.py:282-293) with the O projection done by the persistent
// fp16-output GEMM (o16 = ctx . Wo^T + bo): the residual add and the LayerNorm happen here,
// so the GEMM neither reads nor writes the fp32 stream.  x32 <- LN_prev(x32) + o16 (LN_prev
// rebuilt from the row statistics in `stats` and (pg, pb)), then its statistics and the fp16
// operand image of LN(x32) with (g, b).  fp16 precision mode (kx == 1) only.
template <int NV, bool WX, bool TWO>
__global__ void __launch_bounds__(256)
ln_res_rows_kernel(float* __restrict__ x32, const float2* stats, float2* stats_out, const float* __restrict__ pg,
                   const float* __restrict__ pb, const f16* __restrict__ o16, int rows,
                   const float* __restrict__ g, const float* __restrict__ b, float eps,
                   f16* __restrict__ y16, const float2* __restrict__ stats1, const float* __restrict__ g1,
                   const float* __restrict__ b1, const f16* __restrict__ o16b) {
    constexpr int H = NV * 256;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    const float2 st0 = stats[row];
    float2 st1 = make_float2(0.f, 0.f);
    if constexpr (TWO) st1 = stats1[row];
    float4 x[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int c = v * 256 + lane * 4;
        const float4 r = *(const float4*)(x32 + (size_t)row * H + c);
        const float4 gg = *(const float4*)(pg + c);
        const float4 bb = *(const float4*)(pb + c);
        const half4 o = *(const half4*)(o16 + (size_t)row * H + c);
        x[v] = make_float4(ln_apply(r.x, st0, gg.x, bb.x) + (float)o[0], ln_apply(r.y, st0, gg.y, bb.y) + (float)o[1],
                           ln_apply(r.z, st0, gg.z, bb.z) + (float)o[2], ln_apply(r.w, st0, gg.w, bb.w) + (float)o[3]);
        if constexpr (TWO) {
            // second residual block: x <- LN1(x; st1, g1, b1) + o16b (BertOutput after a deferred
            // BertSelfOutput: x is the post-attention stream the first pass did not store)
            const float4 g4 = *(const float4*)(g1 + c);
            const float4 b4 = *(const float4*)(b1 + c);
            const half4 ob = *(const half4*)(o16b + (size_t)row * H + c);
            x[v] = make_float4(ln_apply(x[v].x, st1, g4.x, b4.x) + (float)ob[0], ln_apply(x[v].y, st1, g4.y, b4.y) + (float)ob[1],
                               ln_apply(x[v].z, st1, g4.z, b4.z) + (float)ob[2], ln_apply(x[v].w, st1, g4.w, b4.w) + (float)ob[3]);
        }
        if constexpr (WX) *(float4*)(x32 + (size_t)row * H + c) = x[v];
    }
    ln_store<NV>(x, g, b, eps, lane, nullptr, stats_out + row, y16 + (size_t)row * H, 1);
}

// BertSelfOutput / BertOutput (modeling_bert.py:282-293, 340-351) in the fp16x3 split-operand
// mode: the projection (x3s GEMM) wrote o32 = dense(h) + bias in fp32; here x = LN_prev(x32) +
// o32 (the residual input rebuilt from the pre-LN stream and its statistics, the reference's
// hidden_states + input_tensor order), x written back as the new pre-LN stream, its statistics,
// and the kx-wide operand image of LN(x) for the next projection.
template <int NV>
__global__ void __launch_bounds__(256)
ln_res32_kernel(float* __restrict__ x32, const float2* stats, float2* stats_out, const float* __restrict__ pg,
                const float* __restrict__ pb, const float* __restrict__ o32, int rows, const float* __restrict__ g,
                const float* __restrict__ b, float eps, f16* __restrict__ y16, int kx) {
    constexpr int H = NV * 256;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    const float2 st0 = stats[row];
    float4 x[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int c = v * 256 + lane * 4;
        const float4 r = *(const float4*)(x32 + (size_t)row * H + c);
        const float4 gg = *(const float4*)(pg + c);
        const float4 bb = *(const float4*)(pb + c);
        const float4 o = *(const float4*)(o32 + (size_t)row * H + c);
        x[v] = make_float4(o.x + ln_apply(r.x, st0, gg.x, bb.x), o.y + ln_apply(r.y, st0, gg.y, bb.y),
                           o.z + ln_apply(r.z, st0, gg.z, bb.z), o.w + ln_apply(r.w, st0, gg.w, bb.w));
        *(float4*)(x32 + (size_t)row * H + c) = x[v];
    }
    ln_store<NV>(x, g, b, eps, lane, nullptr, stats_out + row, y16 + (size_t)row * kx * H, kx);
}

// Residual + LayerNorm of a split-operand layer with the residual stream held ONLY as the
// two-part operand image of the normalised hidden state (h = hi + lo/64, ~22 bits):
//   h16 <- image(LN(o32 + h)), in place (one wave per row reads the whole row first).
// 12 B per element (o32, the image in, the image out) instead of ln_res32's 16 (no fp32
// pre-LN stream, no statistics): the next block's residual is the image itself.
template <int NV>
__global__ void __launch_bounds__(256)
ln_res_img_kernel(f16* __restrict__ h16, const float* __restrict__ o32, int rows, const float* __restrict__ g,
                  const float* __restrict__ b, float eps) {
    constexpr int H = NV * 256;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    f16* hr = h16 + (size_t)row * 2 * H;
    float4 x[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int c = v * 256 + lane * 4;
        const half4 hi = *(const half4*)(hr + il_hi(c)), lo = *(const half4*)(hr + il_hi(c) + 32);
        const float4 o = *(const float4*)(o32 + (size_t)row * H + c);
        x[v] = make_float4(o.x + ((float)hi[0] + (float)lo[0] * X3_DOWN), o.y + ((float)hi[1] + (float)lo[1] * X3_DOWN),
                           o.z + ((float)hi[2] + (float)lo[2] * X3_DOWN), o.w + ((float)hi[3] + (float)lo[3] * X3_DOWN));
    }
    ln_store<NV>(x, g, b, eps, lane, nullptr, nullptr, hr, 2);
}

__device__ __forceinline__ void load8(const f16* p, float (&o)[8]) {
    const half8 v = *(const half8*)p;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (float)v[e];
}
__device__ __forceinline__ void load8(const float* p, float (&o)[8]) {
    const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

// One wave per (sequence, head), one query row per lane, keys in blocks of 64 staged
// in LDS as fp32; online softmax across key blocks (T > 64).
template <class QT>
__global__ void __launch_bounds__(64)
attn_full_kernel(const QT* __restrict__ qkv, SeqMeta sm, int s0, int row0, int H,
                 f16* __restrict__ ctx, int kx, int skip_le) {
    __shared__ __attribute__((aligned(16))) float sK[64][64];
    __shared__ __attribute__((aligned(16))) float sV[64][64];
    const int s = s0 + blockIdx.x, h = blockIdx.y;
    const int T = sm.len[s], rs = sm.row[s] - row0;
    if (T <= skip_le) return;                     // (mixed chunks: the short ones run on MFMA)
    const int lane = threadIdx.x;
    const int ld = 3 * H;
    const QT* base = qkv + (size_t)rs * ld + h * 64;
    const float scale = 0.125f;   // head_dim ** -0.5 with head_dim = 64

    for (int q0 = 0; q0 < T; q0 += 64) {
        const int t = q0 + lane;
        const bool qv = t < T;
        float q[64];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            if (qv) load8(base + (size_t)t * ld + c * 8, v);
#pragma unroll
            for (int e = 0; e < 8; ++e) q[c * 8 + e] = v[e];
        }
        float acc[64];
#pragma unroll
        for (int d = 0; d < 64; ++d) acc[d] = 0.f;
        float m = -INFINITY, l = 0.f;

        for (int k0 = 0; k0 < T; k0 += 64) {
            const int nk = min(64, T - k0);
            __syncthreads();
#pragma unroll
            for (int it = 0; it < 8; ++it) {
                const int kr = it * 8 + (lane >> 3), ch = lane & 7;
                float kv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
                float vv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
                if (kr < nk) {
                    load8(base + (size_t)(k0 + kr) * ld + H + ch * 8, kv);
                    load8(base + (size_t)(k0 + kr) * ld + 2 * H + ch * 8, vv);
                }
                *(float4*)&sK[kr][ch * 8] = make_float4(kv[0], kv[1], kv[2], kv[3]);
                *(float4*)&sK[kr][ch * 8 + 4] = make_float4(kv[4], kv[5], kv[6], kv[7]);
                *(float4*)&sV[kr][ch * 8] = make_float4(vv[0], vv[1], vv[2], vv[3]);
                *(float4*)&sV[kr][ch * 8 + 4] = make_float4(vv[4], vv[5], vv[6], vv[7]);
            }
            __syncthreads();
            float sc[64];
            float bm = -INFINITY;
#pragma unroll
            for (int j = 0; j < 64; ++j) {
                float d0 = 0.f, d1 = 0.f;
                if (j < nk) {
#pragma unroll
                    for (int c = 0; c < 16; c += 2) {
                        const float4 ka = *(const float4*)&sK[j][c * 4];
                        const float4 kb = *(const float4*)&sK[j][c * 4 + 4];
                        d0 += q[c * 4] * ka.x + q[c * 4 + 1] * ka.y + q[c * 4 + 2] * ka.z + q[c * 4 + 3] * ka.w;
                        d1 += q[c * 4 + 4] * kb.x + q[c * 4 + 5] * kb.y + q[c * 4 + 6] * kb.z + q[c * 4 + 7] * kb.w;
                    }
                    sc[j] = (d0 + d1) * scale;
                    bm = fmaxf(bm, sc[j]);
                } else {
                    sc[j] = -INFINITY;
                }
            }
            const float mn = fmaxf(m, bm);
            const float alpha = __expf(m - mn);   // m = -inf on the first block -> 0
            l *= alpha;
#pragma unroll
            for (int d = 0; d < 64; ++d) acc[d] *= alpha;
#pragma unroll
            for (int j = 0; j < 64; ++j) {
                if (j < nk) {
                    const float p = __expf(sc[j] - mn);
                    l += p;
#pragma unroll
                    for (int c = 0; c < 16; ++c) {
                        const float4 vv = *(const float4*)&sV[j][c * 4];
                        acc[c * 4] += p * vv.x;
                        acc[c * 4 + 1] += p * vv.y;
                        acc[c * 4 + 2] += p * vv.z;
                        acc[c * 4 + 3] += p * vv.w;
                    }
                }
            }
            m = mn;
        }
        if (qv) {
            const float il = 1.0f / l;
            f16* o = ctx + (size_t)(rs + t) * kx * H;
#pragma unroll
            for (int c = 0; c < 16; ++c)
                put_split4(o, h * 64 + c * 4, H, kx,
                           make_float4(acc[c * 4] * il, acc[c * 4 + 1] * il, acc[c * 4 + 2] * il, acc[c * 4 + 3] * il));
        }
    }
}

// One wave per (sequence, head), MFMA, latency-lean variant:
//  * K fragments (A operand of X = K.Q^T) go straight from HBM into registers and stay
//    resident across the query tiles (T <= 64: one key block, loaded once);
//  * V is staged ROW-major in LDS with ds_write_b128 and its transposed fragments (A operand
//    of O^T = V^T.P^T) are read with ds_read_b64_tr_b16 (gfx950 hardware transpose): no
//    scalar transposing writes.  V row stride 96 halfs makes those reads conflict-free
//    (the 8 (row, 16-column) blocks of a 32-lane half land on disjoint 8-bank ranges);
//  * all of a key block's global loads are in flight before the first is consumed.
// Numerics: fp16 P, fp32 accumulation, online softmax across 64-key blocks.
// DEDUP (layer 0): qkv holds the chunk's unique rows; position t of sequence s reads row
// urow_m[s] when t is its masked position, urow_h[s] + t otherwise.
template <bool DEDUP>
__global__ void __launch_bounds__(64, 3)
attn_tr_kernel(const f16* __restrict__ qkv, SeqMeta sm, int s0, int row0, int H,
               f16* __restrict__ ctx, int kx) {
    typedef __fp16 fp16x4 __attribute__((__vector_size__(4 * sizeof(__fp16))));
    constexpr int VR = 96;
    __shared__ __attribute__((aligned(16))) f16 sV[64 * VR];
    // grid (sequence, head) (a head-major 1-D grid, the heads of a sequence adjacent, measured
    // 7 % slower, round 1)
    const int s = s0 + (int)blockIdx.x;
    const int hd = (int)blockIdx.y;
    const int T = sm.len[s], rs = sm.row[s] - row0;
    const int lane = threadIdx.x, r = lane & 31, hf = lane >> 5;
    const int ld = 3 * H;
    const int ub = DEDUP ? sm.urow_h[s] : rs;
    const int mp = DEDUP ? sm.mask_pos[s] : -1, um = DEDUP ? sm.urow_m[s] : 0;
    const f16* base = qkv + (size_t)ub * ld + hd * 64;
    const f16* mbase = qkv + (size_t)um * ld + hd * 64;
    // row of position t (the masked copy's [MASK] row lives apart from its hypothesis' rows)
    auto rowp = [&](int t) -> const f16* {
        if constexpr (DEDUP) return t == mp ? mbase : base + (size_t)t * ld;
        else return base + (size_t)t * ld;
    };
    const float scale = 0.125f;                   // head_dim ** -0.5
    const int nkb = (T + 63) >> 6;
    // transposed-read role: 16-lane group g reads keys 4(g>>1) + q (+8), dims 16(g&1) + 4p
    const int g4 = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;
    const int tr_off = (4 * (g4 >> 1) + tq) * VR + 16 * (g4 & 1) + 4 * tp;
    auto tr_read = [&](const f16* p) {
        const fp16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) fp16x4*)p);
        return __builtin_bit_cast(half4, v);
    };

    half8 kf[2][4];
    auto load_kv = [&](int k0) {
        half8 v[8];
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int kr = it * 8 + (lane >> 3), d0 = (lane & 7) * 8;
            v[it] = k0 + kr < T ? *(const half8*)(rowp(k0 + kr) + 2 * H + d0) : (half8){};
        }
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                const int key = k0 + kt * 32 + r;
                kf[kt][ks] = key < T ? *(const half8*)(rowp(key) + H + ks * 16 + hf * 8) : (half8){};
            }
        __syncthreads();                          // previous block's V reads are done
#pragma unroll
        for (int it = 0; it < 8; ++it)
            *(half8*)(sV + (it * 8 + (lane >> 3)) * VR + (lane & 7) * 8) = v[it];
        __syncthreads();
    };

    half8 qn[4];                                  // Q fragments of the next query tile (prefetch)
    auto load_q = [&](int q0) {
        const int t = q0 + r;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
            qn[ks] = t < T ? *(const half8*)(rowp(t) + ks * 16 + hf * 8) : (half8){};
    };
    load_q(0);
    for (int q0 = 0; q0 < T; q0 += 32) {
        const int t = q0 + r;
        half8 qf[4];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) qf[ks] = qn[ks];
        if (q0 + 32 < T) load_q(q0 + 32);
        f32x16 o[2] = {(f32x16){}, (f32x16){}};  // O^T[d tile], lane = query
        float m = -INFINITY, l = 0.f;
        for (int kb = 0; kb < nkb; ++kb) {
            const int k0 = kb * 64;
            if (nkb > 1 || q0 == 0) load_kv(k0);
#pragma unroll
            for (int kt = 0; kt < 2; ++kt) {
                if (k0 + kt * 32 >= T) break;
                f32x16 x = {};
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) x = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf[kt][ks], qf[ks], x, 0, 0, 0);
                float bm = -INFINITY;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const int kj = k0 + kt * 32 + (j & 3) + 8 * (j >> 2) + 4 * hf;
                    const float v = kj < T ? x[j] * scale : -INFINITY;
                    x[j] = v;
                    bm = fmaxf(bm, v);
                }
                bm = fmaxf(bm, __shfl_xor(bm, 32));
                const float mn = fmaxf(m, bm);
                const float alpha = __expf(m - mn);
                half8 pf[2];
                float ls = 0.f;
#pragma unroll
                for (int sk = 0; sk < 2; ++sk)
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const f16 ph = (f16)__expf(x[sk * 8 + e] - mn);
                        pf[sk][e] = ph;
                        ls += (float)ph;
                    }
                ls += __shfl_xor(ls, 32);
                l = l * alpha + ls;
                m = mn;
#pragma unroll
                for (int dt = 0; dt < 2; ++dt) {
#pragma unroll
                    for (int j = 0; j < 16; ++j) o[dt][j] *= alpha;
#pragma unroll
                    for (int sk = 0; sk < 2; ++sk) {
                        // keys kt*32 + 16 sk + 4 hf + {0..3, 8..11}: the P fragment's key order
                        const f16* p = sV + (kt * 32 + 16 * sk) * VR + 32 * dt + tr_off;
                        const half4 lo = tr_read(p), hi = tr_read(p + 8 * VR);
                        const half8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                        o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf, pf[sk], o[dt], 0, 0, 0);
                    }
                }
            }
        }
        if (t < T) {
            const float il = 1.0f / l;
            f16* orow = ctx + (size_t)(rs + t) * kx * H;
#pragma unroll
            for (int dt = 0; dt < 2; ++dt)
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    put_split4(orow, hd * 64 + dt * 32 + 8 * g + 4 * hf, H, kx,
                               make_float4(o[dt][4 * g] * il, o[dt][4 * g + 1] * il,
                                           o[dt][4 * g + 2] * il, o[dt][4 * g + 3] * il));
        }
    }
}

// One wave per (sequence, head) on v_mfma_f32_16x16x32_f16: query tiles of 16 and key tiles
// of 16 (a T = 35 sequence computes 48 x 48 scores instead of 64 x 64 with 32-wide tiles, and
// 12 instead of 16 softmax values per lane and query tile).
//  * Xt = K.Qt per (16-key tile, 16-query tile): lane l holds query l&15, keys 4(l>>4)+e.
//  * softmax over keys: in-lane over the key tiles, then across the 4 lanes of a query
//    (xor 16, 32).
//  * Ot = Vt.Pt per (16-dim tile, 32-key step m): the P fragment is the two key tiles 2m, 2m+1
//    straight from the score registers, so its k index 8(l>>4)+j is key 32m + 4(l>>4) + j
//    (j < 4) or 32m + 16 + 4(l>>4) + j - 4; the Vt fragment follows the same key order with two
//    ds_read_b64_tr_b16 (rows 32m + 4g .. +3 and 32m + 16 + 4g .. +3 of the row-major V image,
//    16 columns).  V row stride 80 halfs: the 8 rows x 16 columns a 32-lane half reads land on
//    disjoint 8-bank ranges.  Vt fragments are read once per key block into registers.
// Online softmax over key blocks of 64 for T > 64.  DEDUP as attn_tr_kernel.
template <bool DEDUP>
__global__ void __launch_bounds__(64, 3)
attn16_kernel(const f16* __restrict__ qkv, SeqMeta sm, int s0, int row0, int H,
              f16* __restrict__ ctx, int kx) {
    typedef __fp16 fp16x4 __attribute__((__vector_size__(4 * sizeof(__fp16))));
    constexpr int VR = 80;
    __shared__ __attribute__((aligned(16))) f16 sV[64 * VR];
    const int s = s0 + blockIdx.x, hd = blockIdx.y;
    const int T = sm.len[s], rs = sm.row[s] - row0;
    const int lane = threadIdx.x, r16 = lane & 15, g = lane >> 4;
    const int ld = 3 * H;
    const int ub = DEDUP ? sm.urow_h[s] : rs;
    const int mp = DEDUP ? sm.mask_pos[s] : -1, um = DEDUP ? sm.urow_m[s] : 0;
    const f16* base = qkv + (size_t)ub * ld + hd * 64;
    const f16* mbase = qkv + (size_t)um * ld + hd * 64;
    auto rowp = [&](int t) -> const f16* {
        if constexpr (DEDUP) return t == mp ? mbase : base + (size_t)t * ld;
        else return base + (size_t)t * ld;
    };
    const float scale = 0.125f;                   // head_dim ** -0.5
    const int nkb = (T + 63) >> 6;
    // transposed-read role: lane 4q+p of group g supplies row 4g + q, columns 4p
    const int tr_off = (4 * g + ((lane & 15) >> 2)) * VR + 4 * (lane & 3);
    auto tr_read = [&](const f16* p) {
        const fp16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) fp16x4*)p);
        return __builtin_bit_cast(half4, v);
    };
    half8 kf[4][2];                               // [key tile][32-dim step]
    half8 vf[4][2];                               // Vt fragments [16-dim tile][32-key step]
    auto load_kv = [&](int k0) {
        half8 v[8];
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int kr = k0 + it * 8 + (lane >> 3);
            v[it] = kr < T ? *(const half8*)(rowp(kr) + 2 * H + (lane & 7) * 8) : (half8){};
        }
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const int key = k0 + kt * 16 + r16;
                kf[kt][ks] = key < T ? *(const half8*)(rowp(key) + H + ks * 32 + g * 8) : (half8){};
            }
        __syncthreads();                          // previous block's V reads are done
#pragma unroll
        for (int it = 0; it < 8; ++it)
            *(half8*)(sV + (it * 8 + (lane >> 3)) * VR + (lane & 7) * 8) = v[it];
        __syncthreads();
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int m2 = 0; m2 < 2; ++m2) {
                const f16* p = sV + (32 * m2) * VR + 16 * dt + tr_off;
                const half4 lo = tr_read(p), hi = tr_read(p + 16 * VR);
                vf[dt][m2] = (half8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            }
    };
    for (int q0 = 0; q0 < T; q0 += 16) {
        const int t = q0 + r16;
        half8 qf[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) qf[ks] = t < T ? *(const half8*)(rowp(t) + ks * 32 + g * 8) : (half8){};
        f32x4 o[4] = {(f32x4){}, (f32x4){}, (f32x4){}, (f32x4){}};   // Ot[16-dim tile], lane = query
        float m = -INFINITY, l = 0.f;
        for (int kb = 0; kb < nkb; ++kb) {
            const int k0 = kb * 64;
            if (nkb > 1 || q0 == 0) load_kv(k0);
            const int nkt = min(4, (T - k0 + 15) >> 4);
            f32x4 x[4];
            float bm = -INFINITY;
#pragma unroll
            for (int kt = 0; kt < 4; ++kt) {
                x[kt] = (f32x4){-INFINITY, -INFINITY, -INFINITY, -INFINITY};
                if (kt < nkt) {
                    f32x4 a = {};
#pragma unroll
                    for (int ks = 0; ks < 2; ++ks) a = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[kt][ks], qf[ks], a, 0, 0, 0);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int key = k0 + kt * 16 + 4 * g + e;
                        const float v = key < T ? a[e] * scale : -INFINITY;
                        x[kt][e] = v;
                        bm = fmaxf(bm, v);
                    }
                }
            }
            bm = fmaxf(bm, __shfl_xor(bm, 16));
            bm = fmaxf(bm, __shfl_xor(bm, 32));
            const float mn = fmaxf(m, bm);
            const float alpha = __expf(m - mn);
            half8 pf[2];
            float ls = 0.f;
#pragma unroll
            for (int m2 = 0; m2 < 2; ++m2)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const f16 ph = (f16)__expf(x[2 * m2 + (j >> 2)][j & 3] - mn);
                    pf[m2][j] = ph;
                    ls += (float)ph;
                }
            ls += __shfl_xor(ls, 16);
            ls += __shfl_xor(ls, 32);
            l = l * alpha + ls;
            m = mn;
            const int nm = (nkt + 1) >> 1;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                o[dt] *= alpha;
#pragma unroll
                for (int m2 = 0; m2 < 2; ++m2)
                    if (m2 < nm) o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf[dt][m2], pf[m2], o[dt], 0, 0, 0);
            }
        }
        if (t < T) {
            const float il = 1.0f / l;
            f16* orow = ctx + (size_t)(rs + t) * kx * H;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
                put_split4(orow, hd * 64 + dt * 16 + 4 * g, H, kx,
                           make_float4(o[dt][0] * il, o[dt][1] * il, o[dt][2] * il, o[dt][3] * il));
        }
    }
}

// fp16x3 precision mode (fp32 Q/K/V from the split-operand QKV GEMM): attn16_kernel's tiling
// with every MFMA operand split into fp16 hi + lo parts and three MFMAs per product
// (hi.hi + hi.lo + lo.hi, the lo.lo term is below fp32 rounding): Xt = K.Qt and Ot = Vt.Pt to
// fp32-level accuracy on the matrix cores instead of the fp32 VALU attention.  The f16 MFMA
// flushes subnormal inputs, and lo = x - hi is subnormal for |x| < 0.25, so lo parts are
// stored scaled by 2^12 (LO_SCALE) and their products go to separate accumulators scaled back
// by 2^-12: 1e-7-level error instead of 3e-5 (tools/diag/attn_split_check.py).  P is split
// after the exponential; the softmax row sum adds the fp32 P.  V is staged as two fp16 images
// (hi, scaled lo).  T <= 64 (one key block; the host routes longer
// sequences to attn_full_kernel<float>).
constexpr float LO_SCALE = 4096.f, LO_UNSCALE = 1.f / 4096.f;
// DEDUP (MLM layer 0): Q, K, V rows come from the chunk's unique rows (row t of copy s is
// unique row urow_m[s] at its masked position, urow_h[s] + t elsewhere), as attn16_kernel.
//
// Layout: V staged for R = 48 or 64 key rows only (R = 48 when
// every sequence of the chunk has T <= 48: the 16 rows past it are zeros the second 32-key
// block reads from registers), 128-B LDS rows without padding — the 16-B chunks XOR-swizzled
// by (row & 6), which keeps the ds_read_b64_tr_b16 lane groups on distinct banks — and the
// Vt fragments read from LDS per query tile instead of held in registers.  R = 48: 12 KiB of
// LDS and <= 168 VGPRs, so 3 waves per SIMD instead of 2.
template <bool DEDUP, int R>
__global__ void __launch_bounds__(64, R == 48 ? 3 : 2)
attn16x3v2_kernel(const float* __restrict__ qkv, SeqMeta sm, int s0, int row0, int H,
                  f16* __restrict__ ctx, int kx) {
    typedef __fp16 fp16x4 __attribute__((__vector_size__(4 * sizeof(__fp16))));
    constexpr int KT = R / 16;                    // 16-key tiles staged
    __shared__ __attribute__((aligned(16))) f16 sVh[R * 64];
    __shared__ __attribute__((aligned(16))) f16 sVl[R * 64];
    const int s = s0 + blockIdx.x, hd = blockIdx.y;
    const int T = sm.len[s], rs = sm.row[s] - row0;
    if (T > R) return;                            // (mixed chunks: the long ones run on attn_full)
    const int lane = threadIdx.x, r16 = lane & 15, g = lane >> 4;
    const int ld = 3 * H;
    const int ub = DEDUP ? sm.urow_h[s] : rs;
    const int mp = DEDUP ? sm.mask_pos[s] : -1, um = DEDUP ? sm.urow_m[s] : 0;
    const float* base = qkv + (size_t)ub * ld + hd * 64;
    const float* mbase = qkv + (size_t)um * ld + hd * 64;
    auto rowp = [&](int t) -> const float* {
        if constexpr (DEDUP) return t == mp ? mbase : base + (size_t)t * ld;
        else return base + (size_t)t * ld;
    };
    // V image address (halfs) of (row, col): 16-B chunk col / 8 swizzled by (row & 6)
    auto vaddr = [](int row, int col) { return row * 64 + ((((col >> 3) ^ (row & 6))) << 3) + (col & 7); };
    const float scale = 0.125f;
    auto tr_read = [&](const f16* p) {
        const fp16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) fp16x4*)p);
        return __builtin_bit_cast(half4, v);
    };
    float4 vraw[R / 4], kraw[KT][2][2];
#pragma unroll
    for (int it = 0; it < R / 4; ++it) {
        const int kr = it * 4 + (lane >> 4), c4 = (lane & 15) * 4;
        vraw[it] = kr < T ? *(const float4*)(rowp(kr) + 2 * H + c4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int key = kt * 16 + r16;
            const float* kp = rowp(key) + H + ks * 32 + g * 8;
            kraw[kt][ks][0] = key < T ? *(const float4*)kp : make_float4(0.f, 0.f, 0.f, 0.f);
            kraw[kt][ks][1] = key < T ? *(const float4*)(kp + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    float4 qraw[2][2];
    auto load_q = [&](int q0) {
        const int t = q0 + r16;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const float* qp = rowp(t) + ks * 32 + g * 8;
            qraw[ks][0] = t < T ? *(const float4*)qp : make_float4(0.f, 0.f, 0.f, 0.f);
            qraw[ks][1] = t < T ? *(const float4*)(qp + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    load_q(0);
    auto split_raw = [](const float4 (&r)[2], half8& hi, half8& lo) {
        const float v[8] = {r[0].x, r[0].y, r[0].z, r[0].w, r[1].x, r[1].y, r[1].z, r[1].w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            hi[e] = (f16)v[e];
            lo[e] = (f16)((v[e] - (float)hi[e]) * LO_SCALE);
        }
    };
#pragma unroll
    for (int it = 0; it < R / 4; ++it) {
        const int kr = it * 4 + (lane >> 4), c4 = (lane & 15) * 4;
        const float4 v = vraw[it];
        const half4 h = {(f16)v.x, (f16)v.y, (f16)v.z, (f16)v.w};
        const half4 l = {(f16)((v.x - (float)h[0]) * LO_SCALE), (f16)((v.y - (float)h[1]) * LO_SCALE),
                         (f16)((v.z - (float)h[2]) * LO_SCALE), (f16)((v.w - (float)h[3]) * LO_SCALE)};
        const int a = vaddr(kr, c4);
        *(half4*)(sVh + a) = h;
        *(half4*)(sVl + a) = l;
    }
    half8 kfh[KT][2], kfl[KT][2];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) split_raw(kraw[kt][ks], kfh[kt][ks], kfl[kt][ks]);
    __syncthreads();
    // transposed-read role: lane supplies row 4g + (l & 15) / 4 of a 16-row group, columns
    // 16 dt + 4 (l & 3); rows 16 and 32 further keep the same swizzle (row & 6)
    const int trow = 4 * g + ((lane & 15) >> 2);
    int tro[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) tro[dt] = vaddr(trow, 16 * dt + 4 * (lane & 3));
    const int nkt = min(KT, (T + 15) >> 4), nm = (nkt + 1) >> 1;
    for (int q0 = 0; q0 < T; q0 += 16) {
        const int t = q0 + r16;
        half8 qh[2], ql[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) split_raw(qraw[ks], qh[ks], ql[ks]);
        if (q0 + 16 < T) load_q(q0 + 16);
        f32x4 x[4];
        float bm = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
            x[kt] = (f32x4){-INFINITY, -INFINITY, -INFINITY, -INFINITY};
            if (kt < KT && kt < nkt) {
                f32x4 a = {}, al = {};
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    al = __builtin_amdgcn_mfma_f32_16x16x32_f16(kfl[kt < KT ? kt : 0][ks], qh[ks], al, 0, 0, 0);
                    al = __builtin_amdgcn_mfma_f32_16x16x32_f16(kfh[kt < KT ? kt : 0][ks], ql[ks], al, 0, 0, 0);
                    a = __builtin_amdgcn_mfma_f32_16x16x32_f16(kfh[kt < KT ? kt : 0][ks], qh[ks], a, 0, 0, 0);
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int key = kt * 16 + 4 * g + e;
                    const float v = key < T ? __builtin_fmaf(al[e], LO_UNSCALE, a[e]) * scale : -INFINITY;
                    x[kt][e] = v;
                    bm = fmaxf(bm, v);
                }
            }
        }
        bm = fmaxf(bm, __shfl_xor(bm, 16));
        bm = fmaxf(bm, __shfl_xor(bm, 32));
        half8 ph[2], pl[2];
        float ls = 0.f;
#pragma unroll
        for (int m2 = 0; m2 < 2; ++m2)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float p = __expf(x[2 * m2 + (j >> 2)][j & 3] - bm);
                ph[m2][j] = (f16)p;
                pl[m2][j] = (f16)((p - (float)ph[m2][j]) * LO_SCALE);
                ls += p;
            }
        ls += __shfl_xor(ls, 16);
        ls += __shfl_xor(ls, 32);
        f32x4 o[4];
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            f32x4 oh = {}, ol = {};
#pragma unroll
            for (int m2 = 0; m2 < 2; ++m2)
                if (m2 < nm) {
                    const int ob = 32 * m2 * 64 + tro[dt];
                    half4 lo = tr_read(sVh + ob), hi = (half4){};
                    if (R == 64 || m2 == 0) hi = tr_read(sVh + ob + 16 * 64);
                    const half8 vh = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    lo = tr_read(sVl + ob);
                    hi = (half4){};
                    if (R == 64 || m2 == 0) hi = tr_read(sVl + ob + 16 * 64);
                    const half8 vl = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    ol = __builtin_amdgcn_mfma_f32_16x16x32_f16(vl, ph[m2], ol, 0, 0, 0);
                    ol = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, pl[m2], ol, 0, 0, 0);
                    oh = __builtin_amdgcn_mfma_f32_16x16x32_f16(vh, ph[m2], oh, 0, 0, 0);
                }
#pragma unroll
            for (int e = 0; e < 4; ++e) o[dt][e] = __builtin_fmaf(ol[e], LO_UNSCALE, oh[e]);
        }
        const float il = 1.0f / ls;
        f16* orow = ctx + (size_t)(rs + t) * kx * H;
        if (kx == 2) {
            // the interleaved image (common.h): lane (r16, g) holds columns 16 dt + 4 g .. + 3 of its
            // query row; one v_permlane16_swap per dword trades the odd lane group's hi parts for the
            // even group's lo parts (rows of 16 lanes: g <-> g ^ 1, the same query row), so every lane
            // stores 8 consecutive halves with one 16-B store — even g: hi of columns 16 dt + 4 g ..
            // + 7, odd g: lo of 16 dt + 4 (g - 1) .. + 7 — instead of two 8-B stores (T21)
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                const float4 v = make_float4(o[dt][0] * il, o[dt][1] * il, o[dt][2] * il, o[dt][3] * il);
                const half4 h = {(f16)v.x, (f16)v.y, (f16)v.z, (f16)v.w};
                const half4 l = {x3_lo(v.x, h[0]), x3_lo(v.y, h[1]), x3_lo(v.z, h[2]), x3_lo(v.w, h[3])};
                const uint2 a = __builtin_bit_cast(uint2, h), b = __builtin_bit_cast(uint2, l);
                const auto r0 = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
                const auto r1 = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
                const int c = hd * 64 + dt * 16 + 4 * (g & ~1);
                if (t < T)
                    *(uint4*)(orow + il_hi(c) + ((g & 1) ? 32 : 0)) = (uint4){r0[0], r1[0], r0[1], r1[1]};
            }
        } else if (t < T) {
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
                put_split4(orow, hd * 64 + dt * 16 + 4 * g, H, kx,
                           make_float4(o[dt][0] * il, o[dt][1] * il, o[dt][2] * il, o[dt][3] * il));
        }
    }
}

// Last layer: one wave per (sequence, head), only the scored query row.  Lanes over keys
// for QK^T, lanes over the 64 head dims for P.V.
template <class QT>
__global__ void __launch_bounds__(64)
attn_query_kernel(const QT* __restrict__ qkv, const QT* __restrict__ qd, const float* __restrict__ x32,
                  const float2* __restrict__ stats, const float* __restrict__ lg,
                  const float* __restrict__ lb, SeqMeta sm, int s0, int row0, int H,
                  f16* __restrict__ ctxq, float* __restrict__ resq, int kx, const f16* __restrict__ himg) {
    __shared__ float sq[64];
    __shared__ float sp[64];
    const int s = s0 + blockIdx.x, h = blockIdx.y;
    const int T = sm.len[s], rs = sm.row[s] - row0, qi = sm.query[s];
    const int lane = threadIdx.x;
    const int ld = 3 * H;
    const QT* base = qkv + (size_t)rs * ld + h * 64;
    // qd: dense [sequence, H] query rows (the last layer projects Q for the scored rows only)
    sq[lane] = (float)(qd ? qd[(size_t)(s - s0) * H + h * 64 + lane] : base[(size_t)qi * ld + lane]) * 0.125f;
    __syncthreads();
    float m = -INFINITY, l = 0.f, acc = 0.f;
    for (int k0 = 0; k0 < T; k0 += 64) {
        const int j = k0 + lane;
        float sc = -INFINITY;
        if (j < T) {
            const QT* kr = base + (size_t)j * ld + H;
            float d = 0.f;
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                float kv[8];
                load8(kr + c * 8, kv);
#pragma unroll
                for (int e = 0; e < 8; ++e) d += sq[c * 8 + e] * kv[e];
            }
            sc = d;
        }
        const float mn = fmaxf(m, wave_max(sc));
        const float p = (j < T) ? __expf(sc - mn) : 0.f;
        const float alpha = __expf(m - mn);
        l = l * alpha + wave_sum(p);
        acc *= alpha;
        __syncthreads();
        sp[lane] = p;
        __syncthreads();
        const int nk = min(64, T - k0);
        for (int jj = 0; jj < nk; ++jj)
            acc += sp[jj] * (float)base[(size_t)(k0 + jj) * ld + 2 * H + lane];
        m = mn;
    }
    const int s_loc = s - s0;
    put_split(ctxq + (size_t)s_loc * kx * H, h * 64 + lane, H, kx, acc / l);
    {   // residual of the scored row: LN of its pre-LN sum, or the normalised state's image
        const int c = h * 64 + lane;
        const size_t r = (size_t)(rs + qi);
        const float2 hl = himg ? il_parts(himg + r * 2 * H, c) : make_float2(0.f, 0.f);
        resq[(size_t)s_loc * H + c] = himg ? hl.x + hl.y * X3_DOWN : ln_apply(x32[r * H + c], stats[r], lg[c], lb[c]);
    }
}

// Row gather: dst[s - s0] = src[row of sequence s's scored position] (ld halfs per row).
__global__ void __launch_bounds__(64)
gather_query_rows_kernel(const f16* __restrict__ src, int ld, SeqMeta sm, int s0, int row0,
                         f16* __restrict__ dst) {
    const int s = s0 + blockIdx.x;
    const size_t r = (size_t)(sm.row[s] - row0 + sm.query[s]);
    const uint4* a = (const uint4*)(src + r * ld);
    uint4* o = (uint4*)(dst + (size_t)blockIdx.x * ld);
    for (int i = threadIdx.x; i < ld / 8; i += 64) o[i] = a[i];
}

__global__ void gather_labels_kernel(const int* __restrict__ tok, SeqMeta sm, int s0, int n,
                                     int* __restrict__ lab) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int s = s0 + i;
    const int l = sm.label[s];
    lab[i] = l >= 0 ? l : tok[sm.tok_off[s] + sm.query[s]];
}

__global__ void __launch_bounds__(256)
lse_finalize_kernel(const float2* __restrict__ part, int n_parts, const float* __restrict__ ll,
                    int rows, float* __restrict__ out) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    const float2* p = part + (size_t)row * n_parts;
    float mx = -INFINITY;
    for (int k = lane; k < n_parts; k += 64)
        if (p[k].y > 0.f) mx = fmaxf(mx, p[k].x);
    mx = wave_max(mx);
    float sm = 0.f;
    for (int k = lane; k < n_parts; k += 64)
        if (p[k].y > 0.f) sm += p[k].y * __expf(p[k].x - mx);
    sm = wave_sum(sm);
    if (lane == 0) out[row] = ll[row] - (mx + logf(sm));
}

__global__ void __launch_bounds__(256)
cls_linear_kernel(const float* __restrict__ h, int rows, int H, const float* __restrict__ w,
                  const float* __restrict__ b, float* __restrict__ out) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    float d = 0.f;
    for (int c = lane; c < H; c += 64) d += h[(size_t)row * H + c] * w[c];
    d = wave_sum(d);
    if (lane == 0) out[row] = d + b[0];
}

__global__ void segsum_f64_kernel(const float* __restrict__ row_lp, const int* __restrict__ off,
                                  int n, double* __restrict__ out) {
    const int h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= n) return;
    double acc = 0.0;
    for (int i = off[h]; i < off[h + 1]; ++i) acc += (double)row_lp[i];
    out[h] = acc;
}

}  // namespace

hipError_t launch_embed_ln(const int* tok, SeqMeta sm, int s0, int s1, int row0, int mask_id,
                           int vocab, const float* word, const float* pos, const float* type0,
                           const float* g, const float* b, float eps, int H, float* x32,
                           float2* stats, f16* h16, int kx, hipStream_t st) {
    const int n = s1 - s0;
    if (n <= 0) return hipSuccess;
#define RS_EMB(NV) hipLaunchKernelGGL(embed_ln_kernel<NV>, dim3(n), dim3(256), 0, st, tok, sm, s0, row0, mask_id, vocab, word, pos, type0, g, b, eps, x32, stats, h16, kx)
    switch (H) {
        case 256: RS_EMB(1); break;
        case 512: RS_EMB(2); break;
        case 768: RS_EMB(3); break;
        case 1024: RS_EMB(4); break;
        default: return hipErrorInvalidValue;
    }
#undef RS_EMB
    return hipGetLastError();
}

hipError_t launch_embed_unique(const int* tok, SeqMeta sm, int s0, int s1, int mask_id, int vocab,
                               const float* word, const float* pos, const float* type0, const float* g,
                               const float* b, float eps, int H, f16* h16u, int kx, hipStream_t st) {
    const int n = s1 - s0;
    if (n <= 0) return hipSuccess;
#define RS_EMBU(NV) hipLaunchKernelGGL(embed_unique_kernel<NV>, dim3(n), dim3(256), 0, st, tok, sm, s0, mask_id, vocab, word, pos, type0, g, b, eps, h16u, kx)
    switch (H) {
        case 256: RS_EMBU(1); break;
        case 512: RS_EMBU(2); break;
        case 768: RS_EMBU(3); break;
        case 1024: RS_EMBU(4); break;
        default: return hipErrorInvalidValue;
    }
#undef RS_EMBU
    return hipGetLastError();
}

// BERTScore embeddings (bert_score bert_encode + greedy_cos_idf's row normalisation):
// e = LN(x) of the last layer, rebuilt from the pre-LN stream, then e / ||e||_2 in fp32,
// stored at the token's position in the caller's ragged token layout: fp16 [H] (TWO false),
// or the two-part image [hi | lo*64] of 2H halves (TWO, the fp16x3 mode: e = hi + lo/64,
// ~22 significant bits, which the split-operand recall kernel multiplies as three products).
template <int NV, bool TWO>
__global__ void __launch_bounds__(256)
embed_out_kernel(const float* __restrict__ x32, const float2* __restrict__ stats,
                 const float* __restrict__ g, const float* __restrict__ b, SeqMeta sm, int s0,
                 int row0, f16* __restrict__ out, const f16* __restrict__ himg) {
    constexpr int H = NV * 256;
    const int s = s0 + blockIdx.x;
    const int T = sm.len[s], rs = sm.row[s] - row0, toff = sm.tok_off[s];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int t = wave; t < T; t += 4) {
        const size_t r = (size_t)(rs + t);
        float4 y[NV];
        float q = 0.f;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const int c = v * 256 + lane * 4;
            if (himg) {                       // the normalised state's (interleaved) two-part image
                const half4 hi = *(const half4*)(himg + r * 2 * H + il_hi(c)), lo = *(const half4*)(himg + r * 2 * H + il_hi(c) + 32);
                y[v] = make_float4((float)hi[0] + (float)lo[0] * X3_DOWN, (float)hi[1] + (float)lo[1] * X3_DOWN,
                                   (float)hi[2] + (float)lo[2] * X3_DOWN, (float)hi[3] + (float)lo[3] * X3_DOWN);
            } else {
                const float2 st = stats[r];
                const float4 x = *(const float4*)(x32 + r * H + c);
                const float4 gg = *(const float4*)(g + c), bb = *(const float4*)(b + c);
                y[v] = make_float4(ln_apply(x.x, st, gg.x, bb.x), ln_apply(x.y, st, gg.y, bb.y),
                                   ln_apply(x.z, st, gg.z, bb.z), ln_apply(x.w, st, gg.w, bb.w));
            }
            q += y[v].x * y[v].x + y[v].y * y[v].y + y[v].z * y[v].z + y[v].w * y[v].w;
        }
        const float nrm = sqrtf(wave_sum(q));
        f16* o = out + (size_t)(toff + t) * H * (TWO ? 2 : 1);
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            const int c = v * 256 + lane * 4;
            const float4 e = make_float4(y[v].x / nrm, y[v].y / nrm, y[v].z / nrm, y[v].w / nrm);
            if constexpr (TWO) {              // the caller's planar [hi | lo*64] layout (rs_token_embed)
                const half4 hi = {(f16)e.x, (f16)e.y, (f16)e.z, (f16)e.w};
                *(half4*)(o + c) = hi;
                *(half4*)(o + H + c) = half4{x3_lo(e.x, hi[0]), x3_lo(e.y, hi[1]), x3_lo(e.z, hi[2]), x3_lo(e.w, hi[3])};
            } else *(half4*)(o + c) = half4{(f16)e.x, (f16)e.y, (f16)e.z, (f16)e.w};
        }
    }
}

hipError_t launch_embed_out(const float* x32, const float2* stats, const float* g, const float* b,
                            SeqMeta sm, int s0, int s1, int row0, int H, f16* out, hipStream_t st, const f16* himg,
                            bool two) {
    const int n = s1 - s0;
    if (n <= 0) return hipSuccess;
#define RS_EO(NV)                                                                                                 \
    do {                                                                                                          \
        if (two) hipLaunchKernelGGL((embed_out_kernel<NV, true>), dim3(n), dim3(256), 0, st, x32, stats, g, b, sm, \
                                    s0, row0, out, himg);                                                         \
        else hipLaunchKernelGGL((embed_out_kernel<NV, false>), dim3(n), dim3(256), 0, st, x32, stats, g, b, sm,   \
                                s0, row0, out, himg);                                                             \
    } while (0)
    switch (H) {
        case 256: RS_EO(1); break;
        case 512: RS_EO(2); break;
        case 768: RS_EO(3); break;
        case 1024: RS_EO(4); break;
        default: return hipErrorInvalidValue;
    }
#undef RS_EO
    return hipGetLastError();
}

hipError_t launch_ln_rows(const float* x, int rows, const float* g, const float* b, float eps,
                          int H, float* y32, float2* stats, f16* y16, int kx, hipStream_t st) {
    if (rows <= 0) return hipSuccess;
    const dim3 grid((rows + 3) / 4);
#define RS_LN(NV) hipLaunchKernelGGL(ln_rows_kernel<NV>, grid, dim3(256), 0, st, x, rows, g, b, eps, y32, stats, y16, kx)
    switch (H) {
        case 256: RS_LN(1); break;
        case 512: RS_LN(2); break;
        case 768: RS_LN(3); break;
        case 1024: RS_LN(4); break;
        default: return hipErrorInvalidValue;
    }
#undef RS_LN
    return hipGetLastError();
}

hipError_t launch_ln_res32(float* x32, const float2* stats, float2* stats_out, const float* pg, const float* pb,
                           const float* o32, int rows, const float* g, const float* b, float eps, int H, f16* y16,
                           int kx, hipStream_t st) {
    if (rows <= 0) return hipSuccess;
    const dim3 grid((rows + 3) / 4), block(256);
#define RS_LN32(NV) hipLaunchKernelGGL(ln_res32_kernel<NV>, grid, block, 0, st, x32, stats, stats_out, pg, pb, o32, \
                                       rows, g, b, eps, y16, kx)
    switch (H) {
        case 256: RS_LN32(1); break;
        case 512: RS_LN32(2); break;
        case 768: RS_LN32(3); break;
        case 1024: RS_LN32(4); break;
        default: return hipErrorInvalidValue;
    }
#undef RS_LN32
    return hipGetLastError();
}

hipError_t launch_ln_res_img(f16* h16, const float* o32, int rows, const float* g, const float* b, float eps, int H,
                             hipStream_t st) {
    if (rows <= 0) return hipSuccess;
    const dim3 grid((rows + 3) / 4), block(256);
#define RS_LNI(NV) hipLaunchKernelGGL(ln_res_img_kernel<NV>, grid, block, 0, st, h16, o32, rows, g, b, eps)
    switch (H) {
        case 256: RS_LNI(1); break;
        case 512: RS_LNI(2); break;
        case 768: RS_LNI(3); break;
        case 1024: RS_LNI(4); break;
        default: return hipErrorInvalidValue;
    }
#undef RS_LNI
    return hipGetLastError();
}

hipError_t launch_ln_res_rows(float* x32, const float2* stats, float2* stats_out, const float* pg, const float* pb,
                             const f16* o16, int rows, const float* g, const float* b, float eps, int H,
                             f16* y16, bool write_x, hipStream_t st, const float2* stats1, const float* g1,
                             const float* b1, const f16* o16b) {
    if (rows <= 0) return hipSuccess;
    const dim3 grid((rows + 3) / 4), block(256);
    const bool two = o16b != nullptr;
    if (two && !write_x) return hipErrorInvalidValue;
#define RS_LNR(NV)                                                                                                   \
    do {                                                                                                             \
        if (two)                                                                                                     \
            hipLaunchKernelGGL((ln_res_rows_kernel<NV, true, true>), grid, block, 0, st, x32, stats, stats_out, pg,  \
                               pb, o16, rows, g, b, eps, y16, stats1, g1, b1, o16b);                                 \
        else if (write_x)                                                                                            \
            hipLaunchKernelGGL((ln_res_rows_kernel<NV, true, false>), grid, block, 0, st, x32, stats, stats_out, pg, \
                               pb, o16, rows, g, b, eps, y16, stats1, g1, b1, o16b);                                 \
        else                                                                                                         \
            hipLaunchKernelGGL((ln_res_rows_kernel<NV, false, false>), grid, block, 0, st, x32, stats, stats_out,    \
                               pg, pb, o16, rows, g, b, eps, y16, stats1, g1, b1, o16b);                             \
    } while (0)
    switch (H) {
        case 256: RS_LNR(1); break;
        case 512: RS_LNR(2); break;
        case 768: RS_LNR(3); break;
        case 1024: RS_LNR(4); break;
        default: return hipErrorInvalidValue;
    }
#undef RS_LNR
    return hipGetLastError();
}

hipError_t launch_attention_full(const void* qkv, bool qkv32, SeqMeta sm, int s0, int s1, int row0,
                                 int H, int heads, f16* ctx, int kx, hipStream_t st, bool dedup, int max_len) {
    if (s1 <= s0) return hipSuccess;
    const dim3 grid(s1 - s0, heads);
    // 16x16x32 tiles while every sequence of the chunk has T <= 64 (longer ones re-stage K/V per
    // 16-query tile: the 32-query tiles of attn_tr_kernel are faster there)
    const bool short16 = max_len > 0 && max_len <= 64;
    auto x3v2 = [&](auto dd) {
        constexpr bool D = decltype(dd)::value;
        if (max_len <= 48)
            hipLaunchKernelGGL((attn16x3v2_kernel<D, 48>), grid, dim3(64), 0, st, (const float*)qkv, sm, s0, row0, H, ctx, kx);
        else
            hipLaunchKernelGGL((attn16x3v2_kernel<D, 64>), grid, dim3(64), 0, st, (const float*)qkv, sm, s0, row0, H, ctx, kx);
    };
    if (dedup && qkv32) {                         // fp16x3 split-operand layer 0 (T <= 64)
        if (kx != 2 || H % 64 || !short16) return hipErrorInvalidValue;
        x3v2(std::true_type{});
        return hipGetLastError();
    }
    if (dedup) {                                  // fp16 QKV, kx == 1 (host gates it)
        if (kx != 1 || H % 64) return hipErrorInvalidValue;
        if (short16) hipLaunchKernelGGL(attn16_kernel<true>, grid, dim3(64), 0, st, (const f16*)qkv, sm, s0, row0, H, ctx, kx);
        else hipLaunchKernelGGL(attn_tr_kernel<true>, grid, dim3(64), 0, st, (const f16*)qkv, sm, s0, row0, H, ctx, kx);
        return hipGetLastError();
    }
    if (qkv32 && short16 && H % 64 == 0) {
        x3v2(std::false_type{});
    } else if (qkv32 && H % 64 == 0) {
        // a chunk with some T > 64: its T <= 64 sequences on the split-MFMA kernel, the longer
        // ones (online softmax over 64-key blocks) on the fp32 VALU kernel; each skips the other's
        hipLaunchKernelGGL((attn16x3v2_kernel<false, 64>), grid, dim3(64), 0, st, (const float*)qkv, sm, s0, row0, H, ctx, kx);
        hipLaunchKernelGGL(attn_full_kernel<float>, grid, dim3(64), 0, st, (const float*)qkv, sm, s0, row0, H, ctx, kx, 64);
    } else if (qkv32) {
        hipLaunchKernelGGL(attn_full_kernel<float>, grid, dim3(64), 0, st, (const float*)qkv, sm, s0, row0, H, ctx, kx, 0);
    } else if (short16) {
        hipLaunchKernelGGL(attn16_kernel<false>, grid, dim3(64), 0, st, (const f16*)qkv, sm, s0, row0, H, ctx, kx);
    } else {
        hipLaunchKernelGGL(attn_tr_kernel<false>, grid, dim3(64), 0, st, (const f16*)qkv, sm, s0, row0, H, ctx, kx);
    }
    return hipGetLastError();
}

hipError_t launch_attention_query(const void* qkv, bool qkv32, const float* x32, const float2* stats,
                                  const float* g, const float* b, SeqMeta sm, int s0, int s1,
                                  int row0, int H, int heads, f16* ctxq, float* resq, int kx,
                                  hipStream_t st, const void* qd, const f16* himg) {
    if (s1 <= s0) return hipSuccess;
    const dim3 grid(s1 - s0, heads);
    if (qkv32)
        hipLaunchKernelGGL(attn_query_kernel<float>, grid, dim3(64), 0, st, (const float*)qkv, (const float*)qd, x32, stats, g, b, sm, s0, row0, H, ctxq, resq, kx, himg);
    else
        hipLaunchKernelGGL(attn_query_kernel<f16>, grid, dim3(64), 0, st, (const f16*)qkv, (const f16*)qd, x32, stats, g, b, sm, s0, row0, H, ctxq, resq, kx, himg);
    return hipGetLastError();
}

hipError_t launch_gather_query_rows(const f16* src, int ld, SeqMeta sm, int s0, int s1, int row0, f16* dst,
                                   hipStream_t st) {
    if (s1 <= s0) return hipSuccess;
    if (ld % 8) return hipErrorInvalidValue;
    hipLaunchKernelGGL(gather_query_rows_kernel, dim3(s1 - s0), dim3(64), 0, st, src, ld, sm, s0, row0, dst);
    return hipGetLastError();
}

hipError_t launch_gather_labels(const int* tok, SeqMeta sm, int s0, int s1, int* lab, hipStream_t st) {
    const int n = s1 - s0;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(gather_labels_kernel, dim3((n + 255) / 256), dim3(256), 0, st, tok, sm, s0, n, lab);
    return hipGetLastError();
}

hipError_t launch_lse_finalize(const float2* part, int n_parts, const float* label_logit, int rows,
                               float* out, hipStream_t st) {
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(lse_finalize_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, part, n_parts, label_logit, rows, out);
    return hipGetLastError();
}

hipError_t launch_cls_linear(const float* h, int rows, int H, const float* w, const float* b,
                             float* out, hipStream_t st) {
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(cls_linear_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, h, rows, H, w, b, out);
    return hipGetLastError();
}

hipError_t launch_segsum_f64(const float* row_lp, const int* hyp_seq_off, int n_hyp, double* out,
                             hipStream_t st) {
    if (n_hyp <= 0) return hipSuccess;
    hipLaunchKernelGGL(segsum_f64_kernel, dim3((n_hyp + 255) / 256), dim3(256), 0, st, row_lp, hyp_seq_off, n_hyp, out);
    return hipGetLastError();
}

// Diagnostic: the memory skeleton of attn_tr_kernel (same Q/K/V reads per (sequence, head)
// wave, ctx written) with no math — the access pattern's own cost.
__global__ void __launch_bounds__(256)
attn_memskel_kernel(const f16* __restrict__ qkv, SeqMeta sm, int H, f16* __restrict__ ctx, int heads_per_block) {
    const int s = blockIdx.x;
    const int T = sm.len[s], rs = sm.row[s];
    const int lane = threadIdx.x & 63, hd = blockIdx.y * heads_per_block + (threadIdx.x >> 6);
    const int ld = 3 * H;
    const f16* base = qkv + (size_t)rs * ld + hd * 64;
    for (int r0 = 0; r0 < T; r0 += 8) {
        const int t = r0 + (lane >> 3), d0 = (lane & 7) * 8;
        if (t < T) {
            const half8 q = *(const half8*)(base + (size_t)t * ld + d0);
            const half8 k = *(const half8*)(base + (size_t)t * ld + H + d0);
            const half8 v = *(const half8*)(base + (size_t)t * ld + 2 * H + d0);
            *(half8*)(ctx + (size_t)(rs + t) * H + hd * 64 + d0) = q + k + v;
        }
    }
}

// Timing/diagnostic entry (not part of the scoring path): one attention launch over
// sequences [0, n_seq) with an explicit kernel kind: 0 attn_tr_kernel, 6 attn16_kernel (fp16
// qkv [rows, 3H], ctx fp16 [rows, H]); 9 attn_full_kernel<float>, 10 / 11 attn16x3v2_kernel with
// 48 / 64 staged key rows (fp32 qkv [rows, 3H], ctx the three-part fp16 image [rows, 3H]);
// 3 / 4 the memory skeleton (one / four heads per block).  len / row: device int32 arrays.
extern "C" int rs_debug_attention(int kind, const void* qkv, const int* len, const int* row, int n_seq,
                                  int H, int heads, void* ctx, void* stream) {
    SeqMeta sm{};
    sm.len = len;
    sm.row = row;
    const dim3 grid(n_seq, heads);
    hipStream_t st = (hipStream_t)stream;
    if (kind == 0)
        hipLaunchKernelGGL(attn_tr_kernel<false>, grid, dim3(64), 0, st, (const f16*)qkv, sm, 0, 0, H, (f16*)ctx, 1);
    else if (kind == 10)
        hipLaunchKernelGGL((attn16x3v2_kernel<false, 48>), grid, dim3(64), 0, st, (const float*)qkv, sm, 0, 0, H, (f16*)ctx, 3);
    else if (kind == 11)
        hipLaunchKernelGGL((attn16x3v2_kernel<false, 64>), grid, dim3(64), 0, st, (const float*)qkv, sm, 0, 0, H, (f16*)ctx, 3);
    else if (kind == 9)
        hipLaunchKernelGGL(attn_full_kernel<float>, grid, dim3(64), 0, st, (const float*)qkv, sm, 0, 0, H, (f16*)ctx, 3, 0);
    else if (kind == 6)
        hipLaunchKernelGGL(attn16_kernel<false>, grid, dim3(64), 0, st, (const f16*)qkv, sm, 0, 0, H, (f16*)ctx, 1);
    else if (kind == 3)
        hipLaunchKernelGGL(attn_memskel_kernel, grid, dim3(64), 0, st, (const f16*)qkv, sm, H, (f16*)ctx, 1);
    else if (kind == 4)
        hipLaunchKernelGGL(attn_memskel_kernel, dim3(n_seq, heads / 4), dim3(256), 0, st, (const f16*)qkv, sm, H, (f16*)ctx, 4);
    else
        return -1;
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

namespace {
// memory skeleton of the two-block ln_res_rows pass: the same loads and stores per row
// (x32 fp32, two fp16 rows, stats; x32 + fp16 image written), no arithmetic beyond a sum
__global__ void __launch_bounds__(256)
lnres_memskel_kernel(float* __restrict__ x32, const f16* __restrict__ o1, const f16* __restrict__ o2, int rows,
                     f16* __restrict__ y16) {
    constexpr int H = 768;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
#pragma unroll
    for (int v = 0; v < 3; ++v) {
        const int c = v * 256 + lane * 4;
        float4 r = *(const float4*)(x32 + (size_t)row * H + c);
        const half4 a = *(const half4*)(o1 + (size_t)row * H + c);
        const half4 b = *(const half4*)(o2 + (size_t)row * H + c);
        r = make_float4(r.x + (float)a[0] + (float)b[0], r.y + (float)a[1] + (float)b[1], r.z + (float)a[2] + (float)b[2],
                        r.w + (float)a[3] + (float)b[3]);
        *(float4*)(x32 + (size_t)row * H + c) = r;
        *(half4*)(y16 + (size_t)row * H + c) = half4{(f16)r.x, (f16)r.y, (f16)r.z, (f16)r.w};
    }
}
}  // namespace

// Timing/diagnostic entry (not part of the scoring path): one LayerNorm-family launch over
// `rows` rows of H = 768.  kind 0 ln_rows, 1 ln_res_rows (x written back), 2 ln_res_rows
// (deferred: stats + image only), 3 two-block ln_res_rows, 4 memory skeleton of kind 3.
extern "C" int rs_debug_ln(int kind, int rows, float* x32, float2* stats, float2* stats1, const void* o1,
                           const void* o2, const float* g, const float* b, void* y16, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    const int H = 768;
    hipError_t e = hipSuccess;
    if (kind == 0) e = launch_ln_rows(x32, rows, g, b, 1e-12f, H, nullptr, stats, (f16*)y16, 1, st);
    else if (kind == 1) e = launch_ln_res_rows(x32, stats, stats, g, b, (const f16*)o1, rows, g, b, 1e-12f, H, (f16*)y16, true, st);
    else if (kind == 2) e = launch_ln_res_rows(x32, stats, stats1, g, b, (const f16*)o1, rows, g, b, 1e-12f, H, (f16*)y16, false, st);
    else if (kind == 3)
        e = launch_ln_res_rows(x32, stats, stats, g, b, (const f16*)o1, rows, g, b, 1e-12f, H, (f16*)y16, true, st, stats1,
                               g, b, (const f16*)o2);
    else {
        hipLaunchKernelGGL(lnres_memskel_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, x32, (const f16*)o1,
                           (const f16*)o2, rows, (f16*)y16);
        e = hipGetLastError();
    }
    return e == hipSuccess ? 0 : -2;
}
