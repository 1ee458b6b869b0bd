// Dependent-chain latency probe (gfx950): one wave, s_memtime around a chain
// of N dependent v_fma_f64 / v_mul_f64 / exp() / ds_read_b64 round trips,
// cycles per step.  Build: hipcc --offload-arch=gfx950 -O3 fp64_latency.hip -o fp64_latency
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ void k(double *out, unsigned long long *cyc, double a, double b, int n)
{
    __shared__ double l[64 * 2];
    double x = a + threadIdx.x * 1e-12;
    l[threadIdx.x] = x;
    l[64 + threadIdx.x] = x;
    __syncthreads();
    unsigned idx = threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
        if (OP == 0) x = fma(x, a, b);
        if (OP == 1) x = x * a;
        if (OP == 2) x = exp(-x * b);
        if (OP == 3) {  // LDS round trip: the address depends on the last value
            x = l[idx];
            idx = (threadIdx.x + (unsigned)(x > 2.0)) & 127u;
        }
        if (OP == 4) x = fma(-a, x, 1.0) * x;  // a Z-row step: fma then mul
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main()
{
    double *out;
    unsigned long long *cyc, h;
    hipMalloc(&out, 64 * sizeof(double));
    hipMalloc(&cyc, sizeof(unsigned long long));
    const char *names[] = {"fma_f64", "mul_f64", "exp(f64)", "ds_read_b64", "fma+mul"};
    const int n = 4096;
    for (int op = 0; op < 5; ++op)
        for (int rep = 0; rep < 3; ++rep) {
            if (op == 0) k<0><<<1, 64>>>(out, cyc, 0.999999, 1e-7, n);
            if (op == 1) k<1><<<1, 64>>>(out, cyc, 0.999999, 1e-7, n);
            if (op == 2) k<2><<<1, 64>>>(out, cyc, 0.5, 1e-3, n);
            if (op == 3) k<3><<<1, 64>>>(out, cyc, 0.5, 1e-3, n);
            if (op == 4) k<4><<<1, 64>>>(out, cyc, 1e-9, 1e-7, n);
            hipDeviceSynchronize();
            hipMemcpy(&h, cyc, sizeof h, hipMemcpyDeviceToHost);
            if (rep == 2) printf("%-12s %.1f s_memtime ticks per dependent step\n", names[op], (double)h / n);
        }
    return 0;
}
