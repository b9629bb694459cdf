// Device helpers shared by the GEMM kernels (k_gemm.hip).
#pragma once
#include "common.h"

namespace {

// Packed GELU for the epilogues: two values per v_pk_* instruction, one transcendental per
// value.  GELU(x) = relu(x) - a * erfc(a / sqrt2) / 2 with a = min(|x|, AMAX), AMAX = 5.7 sqrt2
// (erfc(5.7) < 2e-15: beyond it the term is below fp32 resolution), and erfc(a/sqrt2)/2 = 2^P(a),
// P the degree-6 fit of log2(erfc(a/sqrt2)/2) in a from tools/fit_gelu.py: |GELU error| <= 2.9e-7
// over all x in fp32 (tests/test_gpu_gemm.py::test_gelu_vs_torch_fp32).  Round 6: the polynomial
// is taken in a = |x| itself (the 1/sqrt2 folded into its coefficients, the 1/2 into its constant
// term) and the clamp is one v_min per value with the |x| source modifier — one VALU
// instruction per value fewer than the round-2 form in z = min(|x|/sqrt2, 5.7) (a multiply
// by 1/sqrt2 and one by 1/2); the FFN1 epilogue is VALU-bound (profiles/r6c_stamps.txt: 15 %
// of its tile).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu2(f32x2 x) {
    constexpr float AMAX = 8.06101731f;
    const f32x2 a = __builtin_elementwise_min(__builtin_elementwise_abs(x), (f32x2)(AMAX));
    f32x2 q = __builtin_elementwise_fma(a, (f32x2)(3.309473686e-05f), (f32x2)(-7.692362997e-04f));
    q = __builtin_elementwise_fma(q, a, (f32x2)(8.080770262e-03f));
    q = __builtin_elementwise_fma(q, a, (f32x2)(-5.341218412e-02f));
    q = __builtin_elementwise_fma(q, a, (f32x2)(-4.587709010e-01f));
    q = __builtin_elementwise_fma(q, a, (f32x2)(-1.151201725e+00f));
    q = __builtin_elementwise_fma(q, a, (f32x2)(-9.999930859e-01f));
    const f32x2 e = {__builtin_amdgcn_exp2f(q.x), __builtin_amdgcn_exp2f(q.y)};
    // relu(x) as x - min(x, 0) (exact for every finite x), not max(x, 0): v_min / v_max return the
    // non-NaN operand, so max would turn a NaN pre-activation into 0; this form carries a NaN (and
    // the inf - inf of x = -inf) into the result, where the operand-range guard sees it
    // (rs_api.hip check_finite)
    const f32x2 r = x - __builtin_elementwise_min(x, (f32x2)(0.f));
    return __builtin_elementwise_fma(-a, e, r);
}

// The two-part image's fp16 <-> fp32 steps as v_fma_mix (one instruction per value; hipcc forms
// them only for some of the epilogue's values and otherwise converts with v_cvt_f32_f16 and a
// separate multiply / subtract).  Both are exact rewrites, bitwise equal to the plain forms:
//   mix_val<E>: hi + lo/64 of element E of a packed (hi, lo) fp16 pair — lo/64 is exact, so the
//               fused form rounds once, as (float)hi + (float)lo * (1/64) does;
//   mix_lo2:    RNE(64 x - 64 hi) of a pair into one packed register — 64 (x - hi) is exact in
//               fp32, so the single rounding to fp16 equals x3_lo's.
template <int E>
__device__ __forceinline__ float mix_val(unsigned hi2, unsigned lo2, float inv64) {
    float d;
    if constexpr (E == 0)
        asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(d) : "v"(lo2), "s"(inv64), "v"(hi2));
    else
        asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,1] op_sel_hi:[1,0,1]" : "=v"(d) : "v"(lo2), "s"(inv64), "v"(hi2));
    return d;
}
__device__ __forceinline__ unsigned mix_lo2(unsigned hi2, float x0x64, float x1x64, float neg64) {
    unsigned d;          // mixlo writes the low half (the high half is left for mixhi)
    asm("v_fma_mixlo_f16 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(d) : "v"(hi2), "s"(neg64), "v"(x0x64));
    asm("v_fma_mixhi_f16 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(d) : "v"(hi2), "s"(neg64), "v"(x1x64));
    return d;
}

// 16-byte epilogue store; VAR&64: non-temporal (streamed past L2, keeps the A panels there)
template <int VAR>
__device__ __forceinline__ void st16(uint4* p, uint4 v) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    if constexpr (VAR & 64) __builtin_nontemporal_store((u32x4){v.x, v.y, v.z, v.w}, (u32x4*)p);
    else *p = v;
}

// Chunk swizzle of the split-operand kernel's 64-B LDS rows for 16x16x32 fragment reads: lane
// l reads row r = l & 15 of a 16-aligned block at chunk l >> 4, the ds_read_b128 lane groups
// are {0-3,12-15,20-27}, {4-11,16-19,28-31} and the same + 32; the bank quad of (r, chunk c)
// is 4 (r & 3) + (c ^ g16(r >> 2)), and g16 = [0, 2, 3, 1] makes each group's 16 quads
// distinct (the 32x32 swizzle c ^ ((r >> 2) & 3) collides rows 0-3 with rows 4-7 there).
__device__ __forceinline__ int g16(int rb) { return (0x78 >> (2 * (rb & 3))) & 3; }

// Four 16-B reads of rows rr0 + 8 it (it = 0..3), chunk c16 of a 32 x 128-B epilogue slab whose
// chunks are XOR-swizzled by (row & 7), as inline asm: the compiler treats every LDS read after an
// LDS-DMA issue as a possible alias of the DMA and waits vmcnt(0) first, which would hold each
// epilogue back until the next tile's stage 0 has landed.  The slab is written by this wave's
// own ds_writes just before (LDS ops of a wave execute in order); one lgkmcnt(0) covers the four.
__device__ __forceinline__ void slab_read4(const char* slb, int rr0, int c16, uint4 (&v)[4]) {
    const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)slb;
    uint32_t a[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        const int rr = it * 8 + rr0;
        a[it] = base + rr * 128 + ((c16 ^ (rr & 7)) << 4);
    }
    uint4 v0, v1, v2, v3;
    asm volatile(
        "ds_read_b128 %0, %4\n\t"
        "ds_read_b128 %1, %5\n\t"
        "ds_read_b128 %2, %6\n\t"
        "ds_read_b128 %3, %7\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3)
        : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3])
        : "memory");
    v[0] = v0; v[1] = v1; v[2] = v2; v[3] = v3;
}

}  // namespace
