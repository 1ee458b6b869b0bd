// Latency of one Z-row chain (the fused kernel's and k_qrows' Z value:
// 24 explicit columns in four product chains, the 8-term series by Horner,
// exp) against an ILP-shaped restatement (eight product chains, the series
// by Estrin, exp's polynomial by Estrin), one wave alone on the chip,
// s_memtime around each.  Build: hipcc --offload-arch=gfx950 -O3 zchain_latency.hip -o zchain_latency
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ double exp_estrin(double x)
{
    // x = k ln2 + r, |r| <= ln2 / 2; exp(r) = sum r^i / i!, i <= 11, by Estrin
    const double k = __builtin_rint(x * 1.4426950408889634);
    double r = __builtin_fma(k, -0x1.62e42fefa39efp-1, x);
    r = __builtin_fma(k, -0x1.abc9e3b39803fp-56, r);
    const double r2 = r * r, r4 = r2 * r2, r8 = r4 * r4;
    const double a0 = __builtin_fma(r, 1.0, 1.0), a1 = __builtin_fma(r, 1.0 / 6, 0.5);
    const double a2 = __builtin_fma(r, 1.0 / 120, 1.0 / 24), a3 = __builtin_fma(r, 1.0 / 5040, 1.0 / 720);
    const double a4 = __builtin_fma(r, 1.0 / 362880, 1.0 / 40320), a5 = __builtin_fma(r, 1.0 / 39916800, 1.0 / 3628800);
    const double b0 = __builtin_fma(a1, r2, a0), b1 = __builtin_fma(a3, r2, a2), b2 = __builtin_fma(a5, r2, a4);
    const double p = __builtin_fma(__builtin_fma(b2, r4, b1), r4, b0);
    return __builtin_ldexp(p, (int)k);
    (void)r8;
}

template <int V>
__global__ void k(const double *in, double *out, unsigned long long *cyc, int reps)
{
    __shared__ double sk[32 * 64], zq[8 * 64];
    for (int i = threadIdx.x; i < 32 * 64; i += 64) sk[i] = in[i % 256] * 1e-3;
    for (int i = threadIdx.x; i < 8 * 64; i += 64) zq[i] = in[i % 256] * 1e-5;
    __syncthreads();
    double c = 0.5 + threadIdx.x * 1e-3, acc = 0.0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int rep = 0; rep < reps; ++rep) {
        double s[24], p[8];
#pragma unroll
        for (int i = 0; i < 24; ++i) s[i] = sk[i * 64 + threadIdx.x];
#pragma unroll
        for (int i = 0; i < 8; ++i) p[i] = zq[i * 64 + threadIdx.x];
        double z;
        if (V == 0) {  // the kernels' form
            double za = 1.0, zb = 1.0, zc = 1.0, zd = 1.0;
#pragma unroll
            for (int kk = 0; kk < 24; kk += 8) {
                za *= fma(-c, s[kk + 0], 1.0) * fma(-c, s[kk + 4], 1.0);
                zb *= fma(-c, s[kk + 1], 1.0) * fma(-c, s[kk + 5], 1.0);
                zc *= fma(-c, s[kk + 2], 1.0) * fma(-c, s[kk + 6], 1.0);
                zd *= fma(-c, s[kk + 3], 1.0) * fma(-c, s[kk + 7], 1.0);
            }
            z = (za * zb) * (zc * zd);
            double q = p[7];
#pragma unroll
            for (int i = 6; i >= 0; --i) q = fma(q, c, p[i]);
            z *= exp(-(q * c));
        } else {  // ILP form
            double f[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) f[i] = fma(-c, s[i], 1.0) * fma(-c, s[i + 8], 1.0) * fma(-c, s[i + 16], 1.0);
            z = ((f[0] * f[1]) * (f[2] * f[3])) * ((f[4] * f[5]) * (f[6] * f[7]));
            const double c2 = c * c, c4 = c2 * c2;
            const double q = fma(fma(fma(p[7], c, p[6]), c2, fma(p[5], c, p[4])), c4,
                                 fma(fma(p[3], c, p[2]), c2, fma(p[1], c, p[0])));
            z *= exp_estrin(-(q * c));
        }
        acc += z;
        c = c + acc * 1e-300;  // the next rep depends on this one
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main()
{
    double *in, *out, h_in[256];
    unsigned long long *cyc, h;
    for (int i = 0; i < 256; ++i) h_in[i] = 1.0 + (i * 37 % 101) * 0.01;
    (void)hipMalloc(&in, sizeof h_in);
    (void)hipMalloc(&out, 64 * sizeof(double));
    (void)hipMalloc(&cyc, sizeof h);
    (void)hipMemcpy(in, h_in, sizeof h_in, hipMemcpyHostToDevice);
    const int reps = 256;
    for (int v = 0; v < 2; ++v)
        for (int it = 0; it < 3; ++it) {
            if (v == 0) k<0><<<1, 64>>>(in, out, cyc, reps);
            else k<1><<<1, 64>>>(in, out, cyc, reps);
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(&h, cyc, sizeof h, hipMemcpyDeviceToHost);
            if (it == 2) printf("%s: %.0f cycles per Z row (one wave)\n", v ? "ILP form (8 chains, Estrin)" : "kernels' form", (double)h / reps);
        }
    return 0;
}
