// Issue rate of v_fmac_f64 with a DPP row_newbcast source (gfx950) against
// plain v_fmac_f64 and v_mov_b64: 8 independent accumulators per lane, 4
// waves per SIMD, every SIMD busy.  Why: the DPP-broadcast Q chunks of the
// forward kernels (MDP_JIT_DPPQ) were slower than the
// broadcast LDS reads they replace; this separates the DPP FMA's own cost
// from the zeroed accumulators that variant needs.
// Build: hipcc --offload-arch=gfx950 -O3 dpp_fma_rate.hip -o dpp_fma_rate
#include <hip/hip_runtime.h>
#include <cstdio>

template <int K>
__device__ __forceinline__ double fdpp(double f, double x, double acc)
{
    asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(f), "v"(x), "i"(K));
    return acc;
}
__device__ __forceinline__ double fplain(double f, double x, double acc)
{
    asm volatile("v_fmac_f64_e32 %0, %1, %2" : "+v"(acc) : "v"(f), "v"(x));
    return acc;
}
__device__ __forceinline__ double zero_then_fmac(double f, double x)
{
    double acc;
    asm volatile("v_mov_b64 %0, 0" : "=v"(acc));
    asm volatile("v_fmac_f64_e32 %0, %1, %2" : "+v"(acc) : "v"(f), "v"(x));
    return acc;
}

template <int OP>
__global__ __launch_bounds__(256) void k(double *out, double a, int iters)
{
    double x[8];
    const double f = a + threadIdx.x * 1e-9;
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = a + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (OP == 0) x[i] = fplain(f, a, x[i]);
            if (OP == 1) x[i] = fdpp<3>(f, a, x[i]);
            if (OP == 2) x[i] = zero_then_fmac(f, x[i]);
        }
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main()
{
    const int blocks = 256 * 16, iters = 4096;
    double *out;
    hipMalloc(&out, blocks * 256 * sizeof(double));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[] = {"v_fmac_f64", "v_fmac_f64_dpp row_newbcast", "v_mov_b64 0 + v_fmac_f64"};
    for (int op = 0; op < 3; ++op) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            if (op == 0) k<0><<<blocks, 256>>>(out, 0.999999, iters);
            if (op == 1) k<1><<<blocks, 256>>>(out, 0.999999, iters);
            if (op == 2) k<2><<<blocks, 256>>>(out, 0.999999, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
        }
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double waves = (double)blocks * 4, steps = waves * iters * 8;
        // cycles per step per SIMD at 2.4 GHz: 1024 SIMDs
        printf("%-32s %.3f ms  %.2f SIMD-cycles per wave-step (2.4 GHz)\n", names[op], ms,
               ms * 1e-3 * 2.4e9 * 1024 / steps);
    }
    return 0;
}
