// Issue cost of the instructions the Philox4x32-10 rounds of k_future are
// made of (v_mad_u64_u32, v_xor_b32, v_add_u32) and of v_fma_f64, measured as
// cycles per wave-instruction per SIMD with 8 waves per SIMD and 8
// independent chains per lane (s_memtime around a long unrolled loop).
// Build: hipcc --offload-arch=gfx950 -O3 int_rates.hip -o int_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kIters = 4096, kChains = 8, kBlock = 512;

__global__ __launch_bounds__(kBlock) void k_mad(uint64_t *out, long long *cyc, uint32_t m)
{
    uint32_t lo[kChains], hi[kChains];
    for (int c = 0; c < kChains; ++c) lo[c] = threadIdx.x + c, hi[c] = c;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < kIters; ++i)
#pragma unroll
        for (int c = 0; c < kChains; ++c) {
            const uint64_t p = (uint64_t)lo[c] * m;  // v_mad_u64_u32
            lo[c] = (uint32_t)p ^ hi[c];
            hi[c] = (uint32_t)(p >> 32);
        }
    const long long t1 = __builtin_amdgcn_s_memtime();
    uint64_t s = 0;
    for (int c = 0; c < kChains; ++c) s += lo[c] + hi[c];
    out[blockIdx.x * kBlock + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(kBlock) void k_xor(uint64_t *out, long long *cyc, uint32_t m)
{
    uint32_t a[kChains], b[kChains];
    for (int c = 0; c < kChains; ++c) a[c] = threadIdx.x + c, b[c] = c * m;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < kIters; ++i)
#pragma unroll
        for (int c = 0; c < kChains; ++c) {
            a[c] ^= b[c];
            b[c] += a[c];  // v_add_u32
        }
    const long long t1 = __builtin_amdgcn_s_memtime();
    uint64_t s = 0;
    for (int c = 0; c < kChains; ++c) s += a[c] + b[c];
    out[blockIdx.x * kBlock + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(kBlock) void k_f64(uint64_t *out, long long *cyc, uint32_t m)
{
    double a[kChains];
    for (int c = 0; c < kChains; ++c) a[c] = threadIdx.x + c;
    const double x = 1.0000001 * m;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < kIters; ++i)
#pragma unroll
        for (int c = 0; c < kChains; ++c) a[c] = fma(a[c], x, 0.5);
    const long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
    for (int c = 0; c < kChains; ++c) s += a[c];
    out[blockIdx.x * kBlock + threadIdx.x] = (uint64_t)s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(kBlock) void k_lsh(uint64_t *out, long long *cyc, uint32_t m)
{
    uint64_t a[kChains];
    for (int c = 0; c < kChains; ++c) a[c] = threadIdx.x + c;
    const uint64_t b = m;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < kIters; ++i)
#pragma unroll
        for (int c = 0; c < kChains; ++c) a[c] = (a[c] << 3) + b;  // v_lshl_add_u64
    const long long t1 = __builtin_amdgcn_s_memtime();
    uint64_t s = 0;
    for (int c = 0; c < kChains; ++c) s += a[c];
    out[blockIdx.x * kBlock + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(kBlock) void k_cvt(uint64_t *out, long long *cyc, uint32_t m)
{
    double a[kChains];
    uint32_t u[kChains];
    for (int c = 0; c < kChains; ++c) a[c] = 0.0, u[c] = threadIdx.x + c;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < kIters; ++i)
#pragma unroll
        for (int c = 0; c < kChains; ++c) {
            a[c] += (double)u[c];  // v_cvt_f64_u32 + v_add_f64
            u[c] ^= m;
        }
    const long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
    for (int c = 0; c < kChains; ++c) s += a[c];
    out[blockIdx.x * kBlock + threadIdx.x] = (uint64_t)s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <typename K>
void run(K kernel, const char *name, int insts_per_iter)
{
    const int nb = 256 * 2;  // 2 blocks of 8 waves per CU: 4 waves per SIMD... x2
    uint64_t *out;
    long long *cyc;
    hipMalloc(&out, (size_t)nb * kBlock * 8);
    hipMalloc(&cyc, nb * 8);
    hipLaunchKernelGGL(kernel, dim3(nb), dim3(kBlock), 0, 0, out, cyc, 2654435769u);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kernel, dim3(nb), dim3(kBlock), 0, 0, out, cyc, 2654435769u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    long long c0;
    hipMemcpy(&c0, cyc, 8, hipMemcpyDeviceToHost);
    // per SIMD: nb*kBlock/64 waves over 1024 SIMDs, kIters*kChains*insts each
    const double waves_per_simd = (double)nb * kBlock / 64 / 1024;
    const double wave_insts = waves_per_simd * kIters * kChains * insts_per_iter;
    const double ghz_cycles = ms * 1e-3 * 2.4e9;  // at a nominal 2.4 GHz
    printf("%-28s %8.3f ms  block0 %lld memtime ticks  %.2f cycles/wave-inst at 2.4 GHz\n", name, ms, c0,
           ghz_cycles / wave_insts);
    hipFree(out);
    hipFree(cyc);
}

int main()
{
    run(k_mad, "v_mad_u64_u32 + v_xor", 2);
    run(k_xor, "v_xor + v_add_u32", 2);
    run(k_f64, "v_fma_f64", 1);
    run(k_lsh, "v_lshl_add_u64", 1);
    run(k_cvt, "v_cvt_f64_u32 + v_add_f64 + v_xor", 3);
    return 0;
}
