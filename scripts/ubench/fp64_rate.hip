// FP64 VALU throughput probe (gfx950): v_fma_f64 / v_mul_f64 / v_max_f64 /
// the k_colonise mix, 8 independent chains per lane, enough waves to fill
// every SIMD.  Build: hipcc --offload-arch=gfx950 -O3 fp64_rate.hip -o fp64_rate
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ __launch_bounds__(256) void k(double *out, double a, double b, int iters)
{
    double x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = a + threadIdx.x * 1e-9 + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (OP == 0) x[i] = fma(x[i], a, b);
            if (OP == 1) x[i] = x[i] * a;
            if (OP == 2) x[i] = fmax(x[i], b) + 0.0;
            if (OP == 3) x[i] = x[i] * fmax(0.0, fma(-a, x[i], 1.0));
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
    const char *names[] = {"fma", "mul", "max", "colonise_mix(fma+max+mul)"};
    const int ops[] = {1, 1, 2, 3};  // instructions per element step (max: v_max + v_add folded?)
    for (int op = 0; op < 4; ++op) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            if (op == 0) k<0><<<blocks, 256>>>(out, 0.999999, 1e-7, iters);
            if (op == 1) k<1><<<blocks, 256>>>(out, 0.999999, 1e-7, iters);
            if (op == 2) k<2><<<blocks, 256>>>(out, 0.999999, 1e-7, iters);
            if (op == 3) k<3><<<blocks, 256>>>(out, 1e-9, 1e-7, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
        }
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double lane_steps = (double)blocks * 256 * iters * 8;
        printf("%-28s %.3f ms  %.2f G lane-steps/s  (%.1f per CU-cycle at 2.4 GHz, %d instr/step)\n", names[op], ms,
               lane_steps / ms / 1e6, lane_steps / (ms * 1e-3) / 256 / 2.4e9, ops[op]);
    }
    return 0;
}
