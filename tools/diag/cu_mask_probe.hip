// CU-mask probe (diagnostic, not part of the library): which XCC / SE / CU the workgroups of
// a stream created with hipExtStreamCreateWithCUMask land on, how much HBM bandwidth a
// streaming kernel gets from a subset of the CUs, and whether a compute-bound kernel on the
// complementary mask runs concurrently with it.
//   hipcc -O3 --offload-arch=gfx950 tools/diag/cu_mask_probe.hip -o tools/diag/cu_mask_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <set>
#include <map>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void hwid_kernel(unsigned* out) {
    if (threadIdx.x == 0) {
        // HW_REG_HW_ID (id 4) bits [15:0] and HW_REG_XCC_ID (id 20) bits [3:0]
        const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11));
        const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11));
        out[blockIdx.x] = (xcc << 16) | (hw & 0xffff);
        // keep the block alive a little so blocks spread over the CUs
        long long t0 = clock64();
        while (clock64() - t0 < 20000) {}
    }
}

// float4 copy, grid-stride
__global__ void __launch_bounds__(256) copy_kernel(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = a[i];
}

// U independent float4 loads in flight per thread before the stores
template <int U>
__global__ void __launch_bounds__(256) copy_u_kernel(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += stride * U) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = i + u * stride < n ? a[i + u * stride] : make_float4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < U; ++u) if (i + u * stride < n) b[i + u * stride] = v[u];
    }
}

// compute-bound: FMA chain per thread, one workgroup of 512 threads per CU worth of registers
__global__ void __launch_bounds__(512) fma_kernel(float* out, int iters) {
    float x = threadIdx.x * 1e-3f, y = 1.0001f, z = 0.9999f, w = 0.5f;
    for (int i = 0; i < iters; ++i) {
        x = fmaf(x, y, z); y = fmaf(y, z, w); z = fmaf(z, w, x); w = fmaf(w, x, y);
    }
    if (x + y + z + w == 12345.f) out[0] = x;
}

static hipStream_t masked(const std::vector<int>& cus) {
    uint32_t m[8] = {0};
    for (int c : cus) m[c / 32] |= 1u << (c % 32);
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, 8, m));
    return s;
}

int main() {
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    printf("CUs %d\n", ncu);
    // mem set: bits w*32 + {w, w+8, w+16, w+24} (4 per 32-bit word, residues mod 8 all distinct)
    std::vector<int> mem, gemm;
    std::set<int> ms;
    for (int w = 0; w < 8; ++w) for (int k = 0; k < 4; ++k) ms.insert(w * 32 + w + 8 * k);
    for (int c = 0; c < 256; ++c) (ms.count(c) ? mem : gemm).push_back(c);
    std::vector<int> first32;
    for (int c = 0; c < 32; ++c) first32.push_back(c);
    std::vector<int> every8;
    for (int c = 0; c < 256; c += 8) every8.push_back(c);

    unsigned* d;
    const int NB = 2048;
    CK(hipMalloc(&d, NB * 4));
    std::vector<unsigned> h(NB);
    auto probe = [&](const char* name, hipStream_t s) {
        hipLaunchKernelGGL(hwid_kernel, dim3(NB), dim3(64), 0, s, d);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(h.data(), d, NB * 4, hipMemcpyDeviceToHost));
        std::map<int, std::set<int>> per_xcc;   // xcc -> set of (se, sh, cu)
        for (unsigned v : h) {
            const int xcc = v >> 16, hw = v & 0xffff;
            const int cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
            per_xcc[xcc].insert(se * 32 + sh * 16 + cu);
        }
        printf("%-8s", name);
        int tot = 0;
        for (auto& kv : per_xcc) { printf(" xcc%d:%zu", kv.first, kv.second.size()); tot += kv.second.size(); }
        printf("  total %d CUs\n", tot);
        // block -> xcc pattern of the first 16 blocks
        printf("         first blocks xcc:");
        for (int i = 0; i < 16; ++i) printf(" %u", h[i] >> 16);
        printf("\n");
    };
    hipStream_t s_full, s_mem = masked(mem), s_gemm = masked(gemm), s_f32 = masked(first32), s_e8 = masked(every8);
    CK(hipStreamCreate(&s_full));
    probe("full", s_full);
    probe("mem32", s_mem);
    probe("gemm224", s_gemm);
    probe("first32", s_f32);
    probe("every8", s_e8);

    // bandwidth of a 2 GiB copy (1 GiB read + 1 GiB write) per stream
    const size_t n = (size_t)1 << 26;   // float4 elements = 1 GiB
    float4 *a, *b;
    CK(hipMalloc(&a, n * 16));
    CK(hipMalloc(&b, n * 16));
    CK(hipMemset(a, 0, n * 16));
    float* fo;
    CK(hipMalloc(&fo, 64));
    hipEvent_t e0, e1, e2, e3;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2)); CK(hipEventCreate(&e3));
    auto bw = [&](const char* name, hipStream_t s, int grid) {
        hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(256), 0, s, a, b, n);
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(256), 0, s, a, b, n);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("copy %-8s grid %6d: %.3f ms  %.2f TB/s\n", name, grid, ms / 5, 2.0 * n * 16 / (ms / 5 * 1e-3) / 1e12);
    };
    bw("full", s_full, 8192);
    bw("full", s_full, 2048);
    bw("mem32", s_mem, 256);
    bw("mem32", s_mem, 1024);
    bw("mem32", s_mem, 8192);
    bw("every8", s_e8, 1024);
    auto bwu = [&](const char* name, hipStream_t s, int grid, int U) {
        auto go = [&] {
            if (U == 4) hipLaunchKernelGGL(copy_u_kernel<4>, dim3(grid), dim3(256), 0, s, a, b, n);
            else if (U == 8) hipLaunchKernelGGL(copy_u_kernel<8>, dim3(grid), dim3(256), 0, s, a, b, n);
            else hipLaunchKernelGGL(copy_u_kernel<16>, dim3(grid), dim3(256), 0, s, a, b, n);
        };
        go();
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < 5; ++r) go();
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("copyU%-2d %-8s grid %6d: %.3f ms  %.2f TB/s\n", U, name, grid, ms / 5, 2.0 * n * 16 / (ms / 5 * 1e-3) / 1e12);
    };
    for (int U : {4, 8, 16}) {
        bwu("full", s_full, 2048, U);
        bwu("mem32", s_mem, 256, U);
        bwu("mem32", s_mem, 512, U);
        bwu("first32", s_f32, 512, U);
    }

    // compute kernel alone on gemm224 and full, then concurrently with the copy on mem32
    const int iters = 200000;
    auto tfma = [&](const char* name, hipStream_t s, int grid) {
        hipLaunchKernelGGL(fma_kernel, dim3(grid), dim3(512), 0, s, fo, iters);
        CK(hipEventRecord(e0, s));
        hipLaunchKernelGGL(fma_kernel, dim3(grid), dim3(512), 0, s, fo, iters);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("fma  %-8s grid %6d: %.3f ms\n", name, grid, ms);
        return ms;
    };
    tfma("full", s_full, 256);
    tfma("gemm224", s_gemm, 224);
    // concurrent
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, s_gemm));
    CK(hipEventRecord(e2, s_mem));
    hipLaunchKernelGGL(fma_kernel, dim3(224), dim3(512), 0, s_gemm, fo, iters);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(copy_u_kernel<8>, dim3(512), dim3(256), 0, s_mem, a, b, n);
    CK(hipEventRecord(e1, s_gemm));
    CK(hipEventRecord(e3, s_mem));
    CK(hipDeviceSynchronize());
    float m1, m2;
    CK(hipEventElapsedTime(&m1, e0, e1));
    CK(hipEventElapsedTime(&m2, e2, e3));
    printf("concurrent: fma(gemm224) %.3f ms, 3 copies(mem32) %.3f ms (%.2f TB/s)\n", m1, m2, 3 * 2.0 * n * 16 / (m2 * 1e-3) / 1e12);
    return 0;
}
