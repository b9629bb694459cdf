// Training kernels (RescoreBert distillation training, backward through
// the BERT encoder), with BERT's train-mode dropout (train.h TrDrop).  fp32 throughout — the reference trains in fp32 — with every reduction
// in a fixed order (no float atomics): a training step is bitwise reproducible.
// GEMMs are plain (transposed) fp32 GEMMs on the f32-input MFMA (k_sgemm.hip); everything
// else is here.  One wave per token row for row-wise ops; column reductions in two stages
// (64-row partials, then an ordered sum).
#include "common.h"
#include "train.h"

namespace {

constexpr float kInvSqrt2 = 0.70710678118654752f;
constexpr float kInvSqrt2Pi = 0.39894228040143268f;

template <int NV>
__device__ __forceinline__ void ln_fwd_row(const float4 (&x)[NV], const float* g, const float* b, float eps,
                                           int lane, float2* st, float* h, const TrDrop& dr = TrDrop(),
                                           unsigned long long e0 = 0) {
    constexpr int H = NV * 256;
    float s = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v) s += (x[v].x + x[v].y) + (x[v].z + x[v].w);
    const float mean = wave_sum(s) / (float)H;
    float q = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const float a = x[v].x - mean, bb = x[v].y - mean, c = x[v].z - mean, d = x[v].w - mean;
        q += (a * a + bb * bb) + (c * c + d * d);
    }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)H + eps);
    if (lane == 0) *st = make_float2(mean, rstd);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int c = v * 256 + lane * 4;
        const float4 gg = *(const float4*)(g + c), bb = *(const float4*)(b + c);
        float4 o = make_float4((x[v].x - mean) * rstd * gg.x + bb.x, (x[v].y - mean) * rstd * gg.y + bb.y,
                               (x[v].z - mean) * rstd * gg.z + bb.z, (x[v].w - mean) * rstd * gg.w + bb.w);
        if (dr.thresh)
            o = make_float4(tr_drop(dr, e0 + c, o.x), tr_drop(dr, e0 + c + 1, o.y), tr_drop(dr, e0 + c + 2, o.z),
                            tr_drop(dr, e0 + c + 3, o.w));
        *(float4*)(h + c) = o;
    }
}

// x0 = word[tok] + type[0] + pos[t]; h0 = LN(x0)
template <int NV>
__global__ void __launch_bounds__(256)
tr_embed_ln_kernel(const int* __restrict__ row_tok, const int* __restrict__ row_pos, int M, int vocab,
                   const float* __restrict__ word, const float* __restrict__ pos, const float* __restrict__ type0,
                   const float* __restrict__ g, const float* __restrict__ b, float eps, float* __restrict__ x0,
                   float2* __restrict__ st, float* __restrict__ h0, TrDrop dr) {
    constexpr int H = NV * 256;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= M) return;
    const int id = min(max(row_tok[row], 0), vocab - 1), t = row_pos[row];
    float4 x[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int c = v * 256 + lane * 4;
        const float4 w = *(const float4*)(word + (size_t)id * H + c);
        const float4 ty = *(const float4*)(type0 + c);
        const float4 p = *(const float4*)(pos + (size_t)t * H + c);
        x[v] = make_float4((w.x + ty.x) + p.x, (w.y + ty.y) + p.y, (w.z + ty.z) + p.z, (w.w + ty.w) + p.w);
        *(float4*)(x0 + (size_t)row * H + c) = x[v];
    }
    ln_fwd_row<NV>(x, g, b, eps, lane, st + row, h0 + (size_t)row * H, dr, (unsigned long long)row * H);
}

// y <- drop(y + bias) + res (pre-LN, saved), h = LN(y); bias == nullptr: plain LN of y
template <int NV>
__global__ void __launch_bounds__(256)
tr_bias_res_ln_kernel(float* __restrict__ y, const float* bias, const float* res,
                      int M, const float* __restrict__ g, const float* __restrict__ b, float eps,
                      float2* __restrict__ st, float* __restrict__ h, TrDrop dr) {
    constexpr int H = NV * 256;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= M) return;
    float4 x[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int c = v * 256 + lane * 4;
        x[v] = *(const float4*)(y + (size_t)row * H + c);
        if (bias) {
            const float4 bb = *(const float4*)(bias + c);
            const float4 r = *(const float4*)(res + (size_t)row * H + c);
            float4 o = make_float4(x[v].x + bb.x, x[v].y + bb.y, x[v].z + bb.z, x[v].w + bb.w);
            if (dr.thresh) {
                const unsigned long long e = (unsigned long long)row * H + c;
                o = make_float4(tr_drop(dr, e, o.x), tr_drop(dr, e + 1, o.y), tr_drop(dr, e + 2, o.z),
                                tr_drop(dr, e + 3, o.w));
            }
            x[v] = make_float4(o.x + r.x, o.y + r.y, o.z + r.z, o.w + r.w);
            *(float4*)(y + (size_t)row * H + c) = x[v];
        }
    }
    ln_fwd_row<NV>(x, g, b, eps, lane, st + row, h + (size_t)row * H);
}

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * kInvSqrt2)); }
__device__ __forceinline__ float gelu_erf_grad(float x) {
    return 0.5f * (1.0f + erff(x * kInvSqrt2)) + x * kInvSqrt2Pi * __expf(-0.5f * x * x);
}

// pre <- pre + bias; act = gelu(pre)   (N % 4 == 0)
__global__ void tr_bias_gelu_kernel(float* __restrict__ pre, const float* __restrict__ bias, float* __restrict__ act,
                                    long long n4, int N) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
        const int c = (int)((i * 4) % N);
        float4 v = ((float4*)pre)[i];
        const float4 bb = *(const float4*)(bias + c);
        v = make_float4(v.x + bb.x, v.y + bb.y, v.z + bb.z, v.w + bb.w);
        ((float4*)pre)[i] = v;
        ((float4*)act)[i] = make_float4(gelu_erf(v.x), gelu_erf(v.y), gelu_erf(v.z), gelu_erf(v.w));
    }
}

// dact <- dact * gelu'(pre)
__global__ void tr_gelu_bwd_kernel(float* __restrict__ d, const float* __restrict__ pre, long long n4) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
        float4 v = ((float4*)d)[i];
        const float4 p = ((const float4*)pre)[i];
        ((float4*)d)[i] = make_float4(v.x * gelu_erf_grad(p.x), v.y * gelu_erf_grad(p.y), v.z * gelu_erf_grad(p.z),
                                      v.w * gelu_erf_grad(p.w));
    }
}

__global__ void tr_bias_kernel(float* __restrict__ y, const float* __restrict__ bias, long long n4, int N) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
        const int c = (int)((i * 4) % N);
        float4 v = ((float4*)y)[i];
        const float4 bb = *(const float4*)(bias + c);
        ((float4*)y)[i] = make_float4(v.x + bb.x, v.y + bb.y, v.z + bb.z, v.w + bb.w);
    }
}

// Self-attention forward, one 64-thread block per (sequence, head), thread per query row.
// K and V of the head staged in LDS; P (softmax probabilities) saved for the backward.
// Eager transformers order: scores = (q . k) * scale; softmax = exp(s - max) / sum.
__global__ void __launch_bounds__(64)
tr_attn_fwd_kernel(const float* __restrict__ qkv, const int* __restrict__ seq_off, const int* __restrict__ klen,
                   const long long* __restrict__ pofs, int H, int heads, float* __restrict__ P,
                   float* __restrict__ ctx, TrDrop dr) {
    extern __shared__ __attribute__((aligned(16))) float sm_a[];
    const int s = blockIdx.x, hd = blockIdx.y, tid = threadIdx.x;
    const int r0 = seq_off[s], T = seq_off[s + 1] - r0;
    // keys j >= TK are padding (attention_mask 0): probability exactly 0, as the additive
    // finfo.min mask gives; the backward then carries no gradient to or through them
    const int TK = klen ? min(max(klen[s], 1), T) : T;
    const int ld = 3 * H;
    float* sK = sm_a;                 // [T][64]
    float* sV = sm_a + T * 64;        // [T][64]
    for (int q = tid; q < T * 16; q += 64) {
        const int j = q >> 4, c = (q & 15) * 4;
        const float* rowp = qkv + (size_t)(r0 + j) * ld + hd * 64 + c;
        *(float4*)(sK + j * 64 + c) = *(const float4*)(rowp + H);
        *(float4*)(sV + j * 64 + c) = *(const float4*)(rowp + 2 * H);
    }
    __syncthreads();
    float* Ph = P + pofs[s] + (long long)hd * T * T;
    for (int i = tid; i < T; i += 64) {
        float qv[64];
        const float* qp = qkv + (size_t)(r0 + i) * ld + hd * 64;
#pragma unroll
        for (int c = 0; c < 64; c += 4) {
            const float4 v = *(const float4*)(qp + c);
            qv[c] = v.x; qv[c + 1] = v.y; qv[c + 2] = v.z; qv[c + 3] = v.w;
        }
        float m = -INFINITY;
        for (int j = 0; j < TK; ++j) {
            float d = 0.f;
#pragma unroll
            for (int c = 0; c < 64; ++c) d += qv[c] * sK[j * 64 + c];
            d *= 0.125f;
            Ph[(long long)i * T + j] = d;
            m = fmaxf(m, d);
        }
        for (int j = TK; j < T; ++j) Ph[(long long)i * T + j] = -INFINITY;
        float sum = 0.f;
        for (int j = 0; j < T; ++j) {
            const float e = j < TK ? __expf(Ph[(long long)i * T + j] - m) : 0.f;
            Ph[(long long)i * T + j] = e;
            sum += e;
        }
        float o[64];
#pragma unroll
        for (int c = 0; c < 64; ++c) o[c] = 0.f;
        const unsigned long long e0 = (unsigned long long)(pofs[s] + (long long)hd * T * T + (long long)i * T);
        for (int j = 0; j < T; ++j) {
            const float p = Ph[(long long)i * T + j] / sum;
            Ph[(long long)i * T + j] = p;          // saved before dropout (the backward's P)
            const float pd = tr_drop(dr, e0 + j, p);
#pragma unroll
            for (int c = 0; c < 64; ++c) o[c] += pd * sV[j * 64 + c];
        }
        float* op = ctx + (size_t)(r0 + i) * H + hd * 64;
#pragma unroll
        for (int c = 0; c < 64; c += 4) *(float4*)(op + c) = make_float4(o[c], o[c + 1], o[c + 2], o[c + 3]);
    }
}

// Attention backward per (sequence, head): dP = dctx V^T, dS = P (dP - rowsum(P dP)),
// dq = scale dS K, dk = scale dS^T Q, dv = P^T dctx.  dS lives in LDS.
__global__ void __launch_bounds__(64)
tr_attn_bwd_kernel(const float* __restrict__ qkv, const float* __restrict__ P, const float* __restrict__ dctx,
                   const int* __restrict__ seq_off, const long long* __restrict__ pofs, int H, int heads,
                   float* __restrict__ dqkv, TrDrop dr) {
    extern __shared__ __attribute__((aligned(16))) float sm_a[];
    const int s = blockIdx.x, hd = blockIdx.y, tid = threadIdx.x;
    const int r0 = seq_off[s], T = seq_off[s + 1] - r0;
    const int ld = 3 * H;
    float* sA = sm_a;                 // [T][64]: K (phase 1), Q (phase 2)
    float* sB = sm_a + T * 64;        // [T][64]: V (phase 1), dctx (phase 2)
    float* sS = sm_a + 2 * T * 64;    // [T][T]: dS
    for (int q = tid; q < T * 16; q += 64) {
        const int j = q >> 4, c = (q & 15) * 4;
        const float* rowp = qkv + (size_t)(r0 + j) * ld + hd * 64 + c;
        *(float4*)(sA + j * 64 + c) = *(const float4*)(rowp + H);
        *(float4*)(sB + j * 64 + c) = *(const float4*)(rowp + 2 * H);
    }
    __syncthreads();
    const float* Ph = P + pofs[s] + (long long)hd * T * T;
    for (int i = tid; i < T; i += 64) {
        float g[64];
        const float* gp = dctx + (size_t)(r0 + i) * H + hd * 64;
#pragma unroll
        for (int c = 0; c < 64; c += 4) {
            const float4 v = *(const float4*)(gp + c);
            g[c] = v.x; g[c + 1] = v.y; g[c + 2] = v.z; g[c + 3] = v.w;
        }
        // d(dropped P) = dctx V^T; dP = that * mask * scale
        const unsigned long long e0 = (unsigned long long)(pofs[s] + (long long)hd * T * T + (long long)i * T);
        float rd = 0.f;
        for (int j = 0; j < T; ++j) {
            float d = 0.f;
#pragma unroll
            for (int c = 0; c < 64; ++c) d += g[c] * sB[j * 64 + c];
            d = tr_drop(dr, e0 + j, d);
            sS[i * T + j] = d;
            rd += Ph[(long long)i * T + j] * d;
        }
        float dq[64];
#pragma unroll
        for (int c = 0; c < 64; ++c) dq[c] = 0.f;
        for (int j = 0; j < T; ++j) {
            const float ds = Ph[(long long)i * T + j] * (sS[i * T + j] - rd);
            sS[i * T + j] = ds;
#pragma unroll
            for (int c = 0; c < 64; ++c) dq[c] += ds * sA[j * 64 + c];
        }
        float* o = dqkv + (size_t)(r0 + i) * ld + hd * 64;
#pragma unroll
        for (int c = 0; c < 64; c += 4)
            *(float4*)(o + c) = make_float4(dq[c] * 0.125f, dq[c + 1] * 0.125f, dq[c + 2] * 0.125f, dq[c + 3] * 0.125f);
    }
    __syncthreads();
    for (int q = tid; q < T * 16; q += 64) {
        const int j = q >> 4, c = (q & 15) * 4;
        *(float4*)(sA + j * 64 + c) = *(const float4*)(qkv + (size_t)(r0 + j) * ld + hd * 64 + c);
        *(float4*)(sB + j * 64 + c) = *(const float4*)(dctx + (size_t)(r0 + j) * H + hd * 64 + c);
    }
    __syncthreads();
    for (int j = tid; j < T; j += 64) {
        float dk[64], dv[64];
#pragma unroll
        for (int c = 0; c < 64; ++c) dk[c] = 0.f, dv[c] = 0.f;
        const unsigned long long eb = (unsigned long long)(pofs[s] + (long long)hd * T * T) + j;
        for (int i = 0; i < T; ++i) {
            // dv uses the dropped probabilities the forward multiplied V by
            const float ds = sS[i * T + j], p = tr_drop(dr, eb + (unsigned long long)i * T, Ph[(long long)i * T + j]);
#pragma unroll
            for (int c = 0; c < 64; ++c) {
                dk[c] += ds * sA[i * 64 + c];
                dv[c] += p * sB[i * 64 + c];
            }
        }
        float* o = dqkv + (size_t)(r0 + j) * ld + hd * 64;
#pragma unroll
        for (int c = 0; c < 64; c += 4) {
            *(float4*)(o + H + c) = make_float4(dk[c] * 0.125f, dk[c + 1] * 0.125f, dk[c + 2] * 0.125f, dk[c + 3] * 0.125f);
            *(float4*)(o + 2 * H + c) = make_float4(dv[c], dv[c + 1], dv[c + 2], dv[c + 3]);
        }
    }
}

// LayerNorm backward for one row: dx = rstd (g dy - mean(g dy) - xhat mean(g dy xhat)).
// dx may alias dy.
template <int NV>
__global__ void __launch_bounds__(256)
tr_ln_bwd_kernel(const float* dy, const float* __restrict__ x, const float2* __restrict__ st,
                 const float* __restrict__ g, float* dx, int M) {
    constexpr int H = NV * 256;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= M) return;
    const float2 s = st[row];
    float4 gd[NV], xh[NV];
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int c = v * 256 + lane * 4;
        const float4 d = *(const float4*)(dy + (size_t)row * H + c);
        const float4 xx = *(const float4*)(x + (size_t)row * H + c);
        const float4 gg = *(const float4*)(g + c);
        gd[v] = make_float4(gg.x * d.x, gg.y * d.y, gg.z * d.z, gg.w * d.w);
        xh[v] = make_float4((xx.x - s.x) * s.y, (xx.y - s.x) * s.y, (xx.z - s.x) * s.y, (xx.w - s.x) * s.y);
        a += (gd[v].x + gd[v].y) + (gd[v].z + gd[v].w);
        b += (gd[v].x * xh[v].x + gd[v].y * xh[v].y) + (gd[v].z * xh[v].z + gd[v].w * xh[v].w);
    }
    const float c1 = wave_sum(a) / (float)H, c2 = wave_sum(b) / (float)H;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int c = v * 256 + lane * 4;
        *(float4*)(dx + (size_t)row * H + c) =
            make_float4(s.y * (gd[v].x - c1 - xh[v].x * c2), s.y * (gd[v].y - c1 - xh[v].y * c2),
                        s.y * (gd[v].z - c1 - xh[v].z * c2), s.y * (gd[v].w - c1 - xh[v].w * c2));
    }
}

// Column reductions, stage 1: partial[rb][c] over rows [64 rb, 64 rb + 64) in row order.
//   mode 0: sum dy            (bias grads)
//   mode 1: sum dy * xhat     (LN gamma; xhat from x and (mean, rstd))
constexpr int kRB = 64;
__global__ void tr_colsum_partial_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                         const float2* __restrict__ st, int M, int N, int mode,
                                         float* __restrict__ part) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x, rb = blockIdx.y;
    if (c >= N) return;
    const int r0 = rb * kRB, r1 = min(M, r0 + kRB);
    // four interleaved accumulators (rows r % 4), combined in a fixed order: independent
    // loads in flight, still deterministic
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    if (mode == 0) {
#pragma unroll 8
        for (int r = r0; r < r1; ++r) acc[r & 3] += dy[(size_t)r * N + c];
    } else {
#pragma unroll 4
        for (int r = r0; r < r1; ++r) {
            const float2 s = st[r];
            acc[r & 3] += dy[(size_t)r * N + c] * ((x[(size_t)r * N + c] - s.x) * s.y);
        }
    }
    part[(size_t)rb * N + c] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
}

// Wide form (N % 4 == 0, every training shape): a block of CL column lanes (float4 each, 4 CL
// columns) x 256 / CL row lanes over a row block, row lane l summing rows r0 + l, r0 + l + RL, ...
// in order, the row lanes then combined through LDS in a fixed order (groups of 8 lanes, then the
// groups): 4x the blocks of the form above at a ~1k-token batch, and every lane's loads
// independent.  Rows <= kOnePass: one row block over all rows (CL = 4: 16 columns a block), written
// straight to the output (accumulate: added to it), no second launch; otherwise kRB4-row blocks
// (CL = 16) and the ordered stage 2 below.  MODE 0: part0 = sum dy; 1: part0 = sum dy * xhat; 2:
// both from one read of dy (LayerNorm gamma into part0, beta into part1).
constexpr int kRB4 = 128, kOnePass = 2048;
template <int MODE, bool ONE>
__global__ void __launch_bounds__(256)
tr_colsum4_partial_kernel(const float* __restrict__ dy, const float* __restrict__ x, const float2* __restrict__ st,
                          int M, int N, float* __restrict__ part0, float* __restrict__ part1, int accumulate) {
    constexpr int CL = ONE ? 4 : 16, RL = 256 / CL, NQ = MODE == 2 ? 2 : 1;
    __shared__ float4 red[NQ][RL][CL];
    __shared__ float4 red8[NQ][RL / 8][CL];
    const int cl = threadIdx.x % CL, rl = threadIdx.x / CL;
    const int c = blockIdx.x * 4 * CL + cl * 4, rb = blockIdx.y;
    const int r0 = ONE ? 0 : rb * kRB4, r1 = ONE ? M : min(M, r0 + kRB4);
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    if (c < N) {
#pragma unroll 4
        for (int r = r0 + rl; r < r1; r += RL) {
            const float4 d = *(const float4*)(dy + (size_t)r * N + c);
            if (MODE != 1) {
                b.x += d.x; b.y += d.y; b.z += d.z; b.w += d.w;
            }
            if (MODE != 0) {
                const float2 sr = st[r];
                const float4 xv = *(const float4*)(x + (size_t)r * N + c);
                a.x += d.x * ((xv.x - sr.x) * sr.y);
                a.y += d.y * ((xv.y - sr.x) * sr.y);
                a.z += d.z * ((xv.z - sr.x) * sr.y);
                a.w += d.w * ((xv.w - sr.x) * sr.y);
            }
        }
    }
    red[0][rl][cl] = MODE == 0 ? b : a;
    if (MODE == 2) red[NQ - 1][rl][cl] = b;
    __syncthreads();
    auto add8 = [](const float4* v, int stride) {
        float4 t = v[0];
#pragma unroll
        for (int k = 1; k < 8; ++k) {
            const float4 u = v[k * stride];
            t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
        }
        return t;
    };
    if (rl < RL / 8)
#pragma unroll
        for (int q = 0; q < NQ; ++q) red8[q][rl][cl] = add8(&red[q][8 * rl][cl], CL);
    __syncthreads();
    if (rl == 0 && c < N) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            float4 t = red8[q][0][cl];
#pragma unroll
            for (int k = 1; k < RL / 8; ++k) {
                const float4 v = red8[q][k][cl];
                t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
            }
            float4* o = (float4*)((q == 0 ? part0 : part1) + (size_t)rb * N + c);
            if (ONE && accumulate) {
                const float4 v = *o;
                t.x = v.x + t.x; t.y = v.y + t.y; t.z = v.z + t.z; t.w = v.w + t.w;
            }
            *o = t;
        }
    }
}

// stage 2: out[c] (+)= sum over row blocks in order
__global__ void tr_colsum_final_kernel(const float* __restrict__ part, int nrb, int N, float* __restrict__ out,
                                       int accumulate) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= N) return;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int rb = 0; rb < nrb; ++rb) acc[rb & 3] += part[(size_t)rb * N + c];
    const float a = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    out[c] = accumulate ? out[c] + a : a;
}

// word-embedding gradient: block per distinct token, its rows summed in row order
__global__ void tr_word_grad_kernel(const float* __restrict__ dx0, const int* __restrict__ utok,
                                    const int* __restrict__ toff, const int* __restrict__ rows, int H,
                                    float* __restrict__ dword) {
    const int u = blockIdx.x;
    const int tk = utok[u], a = toff[u], b = toff[u + 1];
    // nn.Embedding(padding_idx = pad_token_id = 0) in BertEmbeddings: the pad id's lookups
    // pass no gradient to its row (the tied MLM decoder's part is added elsewhere)
    if (tk == 0) return;
    for (int c = threadIdx.x; c < H; c += blockDim.x) {
        float acc = 0.f;
        for (int k = a; k < b; ++k) acc += dx0[(size_t)rows[k] * H + c];
        dword[(size_t)tk * H + c] += acc;
    }
}

// position-embedding gradient: block per position, sequences in order
__global__ void tr_pos_grad_kernel(const float* __restrict__ dx0, const int* __restrict__ seq_off, int S, int H,
                                   float* __restrict__ dpos) {
    const int p = blockIdx.x;
    for (int c = threadIdx.x; c < H; c += blockDim.x) {
        float acc = 0.f;
        for (int s = 0; s < S; ++s)
            if (seq_off[s + 1] - seq_off[s] > p) acc += dx0[(size_t)(seq_off[s] + p) * H + c];
        dpos[(size_t)p * H + c] += acc;
    }
}

// RescoreBert head (RescoreBert/model.py:19-20): score_s = h[CLS_s] . w + b
__global__ void tr_cls_fwd_kernel(const float* __restrict__ h, const int* __restrict__ seq_off, int S, int H,
                                  const float* __restrict__ w, const float* __restrict__ b, float* __restrict__ out) {
    const int s = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (s >= S) return;
    const float* hr = h + (size_t)seq_off[s] * H;
    float acc = 0.f;
    for (int c = lane; c < H; c += 64) acc += hr[c] * w[c];
    acc = wave_sum(acc);
    if (lane == 0) out[s] = acc + b[0];
}

// head backward: dh[CLS_s] = dscore_s w (dh zeroed by the caller); dw = sum_s dscore_s h[CLS_s]
// (block per 256 columns, sequences in order); db = sum_s dscore_s
__global__ void tr_cls_bwd_kernel(const float* __restrict__ dsc, const float* __restrict__ h,
                                  const int* __restrict__ seq_off, int S, int H, const float* __restrict__ w,
                                  float* __restrict__ dh, float* __restrict__ dw, float* __restrict__ db) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c < H) {
        float acc = 0.f;
        for (int s = 0; s < S; ++s) {
            const float d = dsc[s];
            acc += d * h[(size_t)seq_off[s] * H + c];
            dh[(size_t)seq_off[s] * H + c] = d * w[c];
        }
        dw[c] += acc;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        float acc = 0.f;
        for (int s = 0; s < S; ++s) acc += dsc[s];
        db[0] += acc;
    }
}

// Distillation losses (single block; groups strided over threads, totals summed by thread 0
// in order).  See train.h for the definitions; every step follows the torch forward /
// autograd sequence of RescoreBert/main.py:104-147 in fp32 (softmax = exp(x - max) / sum,
// log of the softmax OUTPUT for MWED as torch.log(score_distribution) does).
// dsc and uloss are written by one thread and read by another across __syncthreads(): no
// __restrict__ on them, so the compiler cannot move those accesses over the barriers (see
// tr_ce_kernel).
__global__ void tr_loss_kernel(const float* __restrict__ sc, const float* __restrict__ tgt,
                               const float* __restrict__ am, const float* __restrict__ cer,
                               const int* __restrict__ utt_off, int n_utt, int n_hyp, int kind, float md_w,
                               float* dsc, float* uloss, float* __restrict__ loss) {
    const float wmd = kind == RS_LOSS_MD ? 1.0f : md_w;
    for (int h = threadIdx.x; h < n_hyp; h += blockDim.x) dsc[h] = wmd * (2.0f * (sc[h] - tgt[h]));
    __syncthreads();
    if (kind != RS_LOSS_MD) {
        for (int u = threadIdx.x; u < n_utt; u += blockDim.x) {
            const int a = utt_off[u], b = utt_off[u + 1];
            float l = 0.f;
            if (b > a) {
                if (kind == RS_LOSS_MWER) {
                    // P = softmax(mix); MWER_g = sum P (e - sum e / n); d mix = P (d - sum P d)
                    float m = -INFINITY, es = 0.f;
                    for (int i = a; i < b; ++i) { m = fmaxf(m, sc[i] + am[i]); es += cer[i]; }
                    const float avg = es / (float)(b - a);
                    float z = 0.f;
                    for (int i = a; i < b; ++i) z += expf(sc[i] + am[i] - m);
                    for (int i = a; i < b; ++i) l += expf(sc[i] + am[i] - m) / z * (cer[i] - avg);
                    for (int i = a; i < b; ++i) {
                        const float p = expf(sc[i] + am[i] - m) / z;
                        dsc[i] += p * ((cer[i] - avg) - l);
                    }
                } else {
                    // E = softmax(e); T = sum mix / sum e; Q = softmax(mix / T);
                    // KL = sum E (log E - log Q); d z = Q sum E - E; d T = sum d z (-mix / T^2);
                    // d mix = d z / T + d T / sum e
                    float me = -INFINITY, ze = 0.f, smix = 0.f, se = 0.f;
                    for (int i = a; i < b; ++i) { me = fmaxf(me, cer[i]); smix += sc[i] + am[i]; se += cer[i]; }
                    for (int i = a; i < b; ++i) ze += expf(cer[i] - me);
                    const float T = smix / se;
                    float mz = -INFINITY, zq = 0.f;
                    for (int i = a; i < b; ++i) mz = fmaxf(mz, (sc[i] + am[i]) / T);
                    for (int i = a; i < b; ++i) zq += expf((sc[i] + am[i]) / T - mz);
                    float sE = 0.f;
                    for (int i = a; i < b; ++i) sE += expf(cer[i] - me) / ze;
                    float gT = 0.f;
                    for (int i = a; i < b; ++i) {
                        const float mix = sc[i] + am[i];
                        const float E = expf(cer[i] - me) / ze;
                        const float Q = expf(mix / T - mz) / zq;
                        if (E > 0.f) l += E * (logf(E) - logf(Q));
                        const float gz = Q * sE - E;
                        gT += gz * (-mix / (T * T));
                        dsc[i] += gz / T;
                    }
                    for (int i = a; i < b; ++i) dsc[i] += gT / se;
                }
            }
            uloss[u] = l;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float md = 0.f;
        for (int h = 0; h < n_hyp; ++h) md += (sc[h] - tgt[h]) * (sc[h] - tgt[h]);
        float x = 0.f;
        if (kind != RS_LOSS_MD)
            for (int u = 0; u < n_utt; ++u) x += uloss[u];
        loss[0] = kind == RS_LOSS_MD ? md : x + md_w * md;
    }
}

// fixed-tree block reductions (256 threads)
__device__ __forceinline__ float block_reduce(float v, float* sh, bool is_max) {
    const int tid = threadIdx.x;
    sh[tid] = v;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (tid < w) sh[tid] = is_max ? fmaxf(sh[tid], sh[tid + w]) : sh[tid] + sh[tid + w];
        __syncthreads();
    }
    const float r = sh[0];
    __syncthreads();
    return r;
}

// BertForMaskedLM CE (modeling_bert.py:972-975, mean over rows): per row lse - logit[label];
// logits are replaced by d loss / d logits = (softmax - onehot) / M
// The label logit goes through LDS before the first barrier: read from global after the
// reductions (as before), the compiler was free to sink that load past the __syncthreads() that
// precedes the in-place gradient writes (logits was __restrict__), so the row's CE sometimes
// used the thread-(label) gradient instead of the logit — one row's CE off by ~1 in roughly
// one step in four (tools/diag/mlm_first_step.py: 32 of 32 correct after the fix).
__global__ void __launch_bounds__(256)
tr_ce_kernel(float* logits, const int* __restrict__ labels, int M, int V, float* __restrict__ rl) {
    __shared__ float sh[256];
    __shared__ float s_xl;
    const int row = blockIdx.x, tid = threadIdx.x;
    float* x = logits + (size_t)row * V;
    const int lab = min(max(labels[row], 0), V - 1);
    if (tid == 0) s_xl = x[lab];
    float m = -INFINITY;
    for (int j = tid; j < V; j += 256) m = fmaxf(m, x[j]);
    m = block_reduce(m, sh, true);
    float sum = 0.f;
    for (int j = tid; j < V; j += 256) sum += __expf(x[j] - m);
    sum = block_reduce(sum, sh, false);
    const float lse = m + __logf(sum);
    if (tid == 0) rl[row] = lse - s_xl;       // s_xl written before block_reduce's barriers
    __syncthreads();
    const float inv = 1.0f / (float)M;
    for (int j = tid; j < V; j += 256) x[j] = (__expf(x[j] - lse) - (j == lab ? 1.0f : 0.0f)) * inv;
}

__global__ void __launch_bounds__(256) tr_mean_kernel(const float* __restrict__ v, int n, float* __restrict__ out) {
    __shared__ float sh[256];
    float acc = 0.f;
    for (int i = threadIdx.x; i < n; i += 256) acc += v[i];
    acc = block_reduce(acc, sh, false);
    if (threadIdx.x == 0) out[0] = acc / (float)n;
}

// torch.optim.AdamW step (decoupled decay, bias-corrected, exp_avg via lerp)
__global__ void tr_adamw_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                float* __restrict__ v, long long n, float decay, float b1w, float b2, float b2w,
                                float step_size, float bc2_sqrt, float eps) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        float pi = p[i] * decay;
        const float gi = g[i];
        const float mi = m[i] + b1w * (gi - m[i]);
        const float vi = v[i] * b2 + b2w * gi * gi;
        m[i] = mi;
        v[i] = vi;
        const float denom = sqrtf(vi) / bc2_sqrt + eps;
        p[i] = pi - step_size * (mi / denom);
    }
}

// The same update on float4 quads (16-B aligned arrays, n4 = n / 4 quads; the host runs the
// scalar kernel over the n % 4 tail): every element's arithmetic is the scalar kernel's, bit for
// bit, at 16-B accesses (the scalar form moved its 28 B per parameter at ≈ 63 % of HBM peak)
__device__ __forceinline__ float adamw1(float& pi, float gi, float& mi, float& vi, float decay, float b1w, float b2,
                                        float b2w, float step_size, float bc2_sqrt, float eps) {
    pi *= decay;
    mi = mi + b1w * (gi - mi);
    vi = vi * b2 + b2w * gi * gi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    pi = pi - step_size * (mi / denom);
    return pi;
}
__global__ void tr_adamw4_kernel(float4* __restrict__ p, const float4* __restrict__ g, float4* __restrict__ m,
                                 float4* __restrict__ v, long long n4, float decay, float b1w, float b2, float b2w,
                                 float step_size, float bc2_sqrt, float eps) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
        float4 pi = p[i], mi = m[i], vi = v[i];
        const float4 gi = g[i];
        adamw1(pi.x, gi.x, mi.x, vi.x, decay, b1w, b2, b2w, step_size, bc2_sqrt, eps);
        adamw1(pi.y, gi.y, mi.y, vi.y, decay, b1w, b2, b2w, step_size, bc2_sqrt, eps);
        adamw1(pi.z, gi.z, mi.z, vi.z, decay, b1w, b2, b2w, step_size, bc2_sqrt, eps);
        adamw1(pi.w, gi.w, mi.w, vi.w, decay, b1w, b2, b2w, step_size, bc2_sqrt, eps);
        m[i] = mi;
        v[i] = vi;
        p[i] = pi;
    }
}

__global__ void tr_dropout_kernel(float* dst, const float* src, long long n, TrDrop dr) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        dst[i] = tr_drop(dr, (unsigned long long)i, src[i]);
}

__global__ void tr_dropout_keep_kernel(uint8_t* __restrict__ keep, long long n, TrDrop dr) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        keep[i] = dr.thresh == 0 ? 1 : (uint8_t)tr_keep(dr, (unsigned long long)i);
}

int grid_for(long long n, int bs) { return (int)std::min<long long>((n + bs - 1) / bs, 8192); }

}  // namespace

#define RS_NV_SWITCH(H, CALL)                \
    switch (H) {                             \
        case 256: { constexpr int NV = 1; CALL; } break;  \
        case 512: { constexpr int NV = 2; CALL; } break;  \
        case 768: { constexpr int NV = 3; CALL; } break;  \
        case 1024: { constexpr int NV = 4; CALL; } break; \
        default: return hipErrorInvalidValue; \
    }

hipError_t tr_embed_ln(const int* row_tok, const int* row_pos, int M, int vocab, const float* word,
                       const float* pos, const float* type0, const float* g, const float* b, float eps, int H,
                       float* x0, float2* st, float* h0, hipStream_t s, const TrDrop& d) {
    if (M <= 0) return hipSuccess;
    RS_NV_SWITCH(H, hipLaunchKernelGGL(tr_embed_ln_kernel<NV>, dim3((M + 3) / 4), dim3(256), 0, s, row_tok, row_pos,
                                       M, vocab, word, pos, type0, g, b, eps, x0, st, h0, d));
    return hipGetLastError();
}

hipError_t tr_bias_res_ln(float* y, const float* bias, const float* res, int M, const float* g, const float* b,
                          float eps, int H, float2* st, float* h, hipStream_t s, const TrDrop& d) {
    if (M <= 0) return hipSuccess;
    RS_NV_SWITCH(H, hipLaunchKernelGGL(tr_bias_res_ln_kernel<NV>, dim3((M + 3) / 4), dim3(256), 0, s, y, bias, res,
                                       M, g, b, eps, st, h, bias ? d : TrDrop()));
    return hipGetLastError();
}

hipError_t tr_bias_gelu(float* pre, const float* bias, float* act, int M, int N, hipStream_t s) {
    const long long n4 = (long long)M * N / 4;
    if (n4 <= 0) return hipSuccess;
    hipLaunchKernelGGL(tr_bias_gelu_kernel, dim3(grid_for(n4, 256)), dim3(256), 0, s, pre, bias, act, n4, N);
    return hipGetLastError();
}

hipError_t tr_gelu_bwd(float* d, const float* pre, long long n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(tr_gelu_bwd_kernel, dim3(grid_for(n / 4, 256)), dim3(256), 0, s, d, pre, n / 4);
    return hipGetLastError();
}

hipError_t tr_bias(float* y, const float* bias, int M, int N, hipStream_t s) {
    const long long n4 = (long long)M * N / 4;
    if (n4 <= 0) return hipSuccess;
    hipLaunchKernelGGL(tr_bias_kernel, dim3(grid_for(n4, 256)), dim3(256), 0, s, y, bias, n4, N);
    return hipGetLastError();
}

static size_t attn_smem(int tmax, bool bwd) { return (size_t)(2 * tmax * 64 + (bwd ? tmax * tmax : 0)) * 4; }

hipError_t tr_attn_fwd(const float* qkv, const int* seq_off, const int* klen, const long long* pofs, int S,
                       int tmax, int H, int heads, float* P, float* ctx, hipStream_t s, const TrDrop& d) {
    if (S <= 0) return hipSuccess;
    const size_t sm = attn_smem(tmax, false);
    hipError_t e = hipFuncSetAttribute((const void*)tr_attn_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(tr_attn_fwd_kernel, dim3(S, heads), dim3(64), sm, s, qkv, seq_off, klen, pofs, H, heads, P, ctx, d);
    return hipGetLastError();
}

hipError_t tr_attn_bwd(const float* qkv, const float* P, const float* dctx, const int* seq_off, const long long* pofs,
                       int S, int tmax, int H, int heads, float* dqkv, hipStream_t s, const TrDrop& d) {
    if (S <= 0) return hipSuccess;
    const size_t sm = attn_smem(tmax, true);
    hipError_t e = hipFuncSetAttribute((const void*)tr_attn_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(tr_attn_bwd_kernel, dim3(S, heads), dim3(64), sm, s, qkv, P, dctx, seq_off, pofs, H, heads, dqkv, d);
    return hipGetLastError();
}

hipError_t tr_ln_bwd(const float* dy, const float* x, const float2* st, const float* g, float* dx, int M, int H,
                     hipStream_t s) {
    if (M <= 0) return hipSuccess;
    RS_NV_SWITCH(H, hipLaunchKernelGGL(tr_ln_bwd_kernel<NV>, dim3((M + 3) / 4), dim3(256), 0, s, dy, x, st, g, dx, M));
    return hipGetLastError();
}

// floats: the kRB-row partials of tr_colsum's narrow form, or two arrays of kRB4-row partials
size_t tr_colsum_scratch(int M, int N) {
    return std::max((size_t)((M + kRB - 1) / kRB), (size_t)2 * ((M + kRB4 - 1) / kRB4)) * N * 4;
}

hipError_t tr_colsum(const float* dy, const float* x, const float2* st, int M, int N, int mode, float* part,
                     float* out, int accumulate, hipStream_t s) {
    if (M <= 0 || N <= 0) return hipSuccess;
    if (N % 4 == 0) {
        const dim3 g1((N + 63) / 64), g16((N + 15) / 16);
        if (M <= kOnePass) {
            if (mode == 0)
                hipLaunchKernelGGL((tr_colsum4_partial_kernel<0, true>), g16, dim3(256), 0, s, dy, x, st, M, N, out, out, accumulate);
            else
                hipLaunchKernelGGL((tr_colsum4_partial_kernel<1, true>), g16, dim3(256), 0, s, dy, x, st, M, N, out, out, accumulate);
            return hipGetLastError();
        }
        const int nrb = (M + kRB4 - 1) / kRB4;
        if (mode == 0)
            hipLaunchKernelGGL((tr_colsum4_partial_kernel<0, false>), dim3(g1.x, nrb), dim3(256), 0, s, dy, x, st, M, N, part, part, 0);
        else
            hipLaunchKernelGGL((tr_colsum4_partial_kernel<1, false>), dim3(g1.x, nrb), dim3(256), 0, s, dy, x, st, M, N, part, part, 0);
        hipLaunchKernelGGL(tr_colsum_final_kernel, g1, dim3(64), 0, s, part, nrb, N, out, accumulate);
        return hipGetLastError();
    }
    const int nrb = (M + kRB - 1) / kRB;
    hipLaunchKernelGGL(tr_colsum_partial_kernel, dim3((N + 255) / 256, nrb), dim3(256), 0, s, dy, x, st, M, N, mode, part);
    hipLaunchKernelGGL(tr_colsum_final_kernel, dim3((N + 63) / 64), dim3(64), 0, s, part, nrb, N, out, accumulate);
    return hipGetLastError();
}

// LayerNorm gamma (sum dy * xhat) and beta (sum dy) gradients from one read of dy: the two
// tr_colsum calls' results bit for bit (the same per-column order), half the dy reads and launches
hipError_t tr_colsum_ln(const float* dy, const float* x, const float2* st, int M, int N, float* part, float* out_g,
                        float* out_b, hipStream_t s) {
    if (M <= 0 || N <= 0) return hipSuccess;
    if (N % 4) {
        if (hipError_t e = tr_colsum(dy, x, st, M, N, 1, part, out_g, 0, s)) return e;
        return tr_colsum(dy, nullptr, nullptr, M, N, 0, part, out_b, 0, s);
    }
    if (M <= kOnePass) {
        hipLaunchKernelGGL((tr_colsum4_partial_kernel<2, true>), dim3((N + 15) / 16), dim3(256), 0, s, dy, x, st, M, N, out_g,
                           out_b, 0);
        return hipGetLastError();
    }
    const int nrb = (M + kRB4 - 1) / kRB4;
    float* part_b = part + (size_t)nrb * N;         // tr_colsum_scratch: room for two
    hipLaunchKernelGGL((tr_colsum4_partial_kernel<2, false>), dim3((N + 63) / 64, nrb), dim3(256), 0, s, dy, x, st, M, N, part,
                       part_b, 0);
    hipLaunchKernelGGL(tr_colsum_final_kernel, dim3((N + 63) / 64), dim3(64), 0, s, part, nrb, N, out_g, 0);
    hipLaunchKernelGGL(tr_colsum_final_kernel, dim3((N + 63) / 64), dim3(64), 0, s, part_b, nrb, N, out_b, 0);
    return hipGetLastError();
}

hipError_t tr_word_grad(const float* dx0, const int* utok, const int* toff, const int* rows, int n_uniq, int H,
                        float* dword, hipStream_t s) {
    if (n_uniq <= 0) return hipSuccess;
    hipLaunchKernelGGL(tr_word_grad_kernel, dim3(n_uniq), dim3(256), 0, s, dx0, utok, toff, rows, H, dword);
    return hipGetLastError();
}

hipError_t tr_pos_grad(const float* dx0, const int* seq_off, int S, int tmax, int H, float* dpos, hipStream_t s) {
    if (S <= 0 || tmax <= 0) return hipSuccess;
    hipLaunchKernelGGL(tr_pos_grad_kernel, dim3(tmax), dim3(256), 0, s, dx0, seq_off, S, H, dpos);
    return hipGetLastError();
}

hipError_t tr_cls_fwd(const float* h, const int* seq_off, int S, int H, const float* w, const float* b, float* out,
                      hipStream_t s) {
    if (S <= 0) return hipSuccess;
    hipLaunchKernelGGL(tr_cls_fwd_kernel, dim3((S + 3) / 4), dim3(256), 0, s, h, seq_off, S, H, w, b, out);
    return hipGetLastError();
}

hipError_t tr_cls_bwd(const float* dsc, const float* h, const int* seq_off, int S, int H, const float* w, float* dh,
                      float* dw, float* db, hipStream_t s) {
    hipLaunchKernelGGL(tr_cls_bwd_kernel, dim3((H + 255) / 256), dim3(256), 0, s, dsc, h, seq_off, S, H, w, dh, dw, db);
    return hipGetLastError();
}

hipError_t tr_loss(const float* sc, const float* tgt, const float* am, const float* err, const int* utt_off,
                   int n_utt, int n_hyp, int kind, float md_w, float* dsc, float* uloss, float* loss, hipStream_t s) {
    hipLaunchKernelGGL(tr_loss_kernel, dim3(1), dim3(256), 0, s, sc, tgt, am, err, utt_off, n_utt, n_hyp, kind, md_w,
                       dsc, uloss, loss);
    return hipGetLastError();
}

hipError_t tr_ce(float* logits, const int* labels, int M, int V, float* row_loss, float* loss, hipStream_t s) {
    if (M <= 0) return hipSuccess;
    hipLaunchKernelGGL(tr_ce_kernel, dim3(M), dim3(256), 0, s, logits, labels, M, V, row_loss);
    hipLaunchKernelGGL(tr_mean_kernel, dim3(1), dim3(256), 0, s, row_loss, M, loss);
    return hipGetLastError();
}

hipError_t tr_adamw(float* p, const float* g, float* m, float* v, long long n, float decay, float b1w, float b2,
                    float b2w, float step_size, float bc2_sqrt, float eps, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if ((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0 && n >= 4) {
        const long long n4 = n / 4, done = n4 * 4;
        hipLaunchKernelGGL(tr_adamw4_kernel, dim3(grid_for(n4, 256)), dim3(256), 0, s, (float4*)p, (const float4*)g,
                           (float4*)m, (float4*)v, n4, decay, b1w, b2, b2w, step_size, bc2_sqrt, eps);
        if (done < n)
            hipLaunchKernelGGL(tr_adamw_kernel, dim3(1), dim3(64), 0, s, p + done, g + done, m + done, v + done, n - done,
                               decay, b1w, b2, b2w, step_size, bc2_sqrt, eps);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(tr_adamw_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, p, g, m, v, n, decay, b1w, b2, b2w,
                       step_size, bc2_sqrt, eps);
    return hipGetLastError();
}

hipError_t tr_dropout(float* dst, const float* src, long long n, const TrDrop& d, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(tr_dropout_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, dst, src, n, d);
    return hipGetLastError();
}

hipError_t tr_dropout_keep(uint8_t* keep, long long n, const TrDrop& d, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(tr_dropout_keep_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, keep, n, d);
    return hipGetLastError();
}
