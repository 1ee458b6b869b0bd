// Per-dispatch overhead against the workgroup shape: a 256-block kernel of
// fixed duration launched back to back with 256 / 512 / 1024 threads per
// block and 0 / 40 / 150 KiB of dynamic LDS (the engine's kernels run 1 024
// threads with up to 150 KiB).  Prints the mean launch-to-launch time, the
// blocks' wall span (s_memrealtime, 100 MHz) and the difference.
// Build: hipcc --offload-arch=gfx950 -O3 launch_shape.hip -o launch_shape
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(1024) void k_shape(unsigned long long *t, double *out, int iters)
{
    extern __shared__ double lds[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    double a = threadIdx.x * 1e-3, b = 1.0;
    for (int k = 0; k < iters; ++k) {
        a = fma(a, 0.999999, 1e-7);
        b = fma(b, 1.000001, -1e-7);
    }
    lds[threadIdx.x] = a;
    __syncthreads();
    // one coalesced store per lane, 8 B x threads per block
    out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = lds[blockDim.x - 1 - threadIdx.x] + b;
    if (threadIdx.x == 0) {
        t[2 * blockIdx.x] = t0;
        t[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

int main()
{
    const int nb = 256, N = 200;
    unsigned long long *t;
    double *out;
    hipMalloc(&t, 2 * nb * 8);
    hipMalloc(&out, (size_t)nb * 1024 * 8);
    hipFuncSetAttribute((const void *)k_shape, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<unsigned long long> h(2 * nb);
    for (int threads : {256, 512, 1024})
        for (int kib : {0, 40, 150}) {
            const int iters = 300 * 512 / threads;  // about the same block duration
            const size_t dyn = (size_t)kib * 1024 + 8 * 1024;
            auto launch = [&]() { hipLaunchKernelGGL(k_shape, dim3(nb), dim3(threads), dyn, s, t, out, iters); };
            for (int i = 0; i < 20; ++i) launch();
            hipStreamSynchronize(s);
            hipEventRecord(e0, s);
            for (int i = 0; i < N; ++i) launch();
            hipEventRecord(e1, s);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            hipMemcpy(h.data(), t, 2 * nb * 8, hipMemcpyDeviceToHost);
            unsigned long long lo = ~0ull, hi = 0;
            for (int b = 0; b < nb; ++b) {
                lo = std::min(lo, h[2 * b]);
                hi = std::max(hi, h[2 * b + 1]);
            }
            const double per = ms * 1e3 / N, wall = (hi - lo) * 0.01;
            printf("threads %4d  dyn LDS %3d+8 KiB: per-launch %6.2f us  block wall %6.2f us  outside %5.2f us\n", threads,
                   kib, per, wall, per - wall);
        }
    return 0;
}
