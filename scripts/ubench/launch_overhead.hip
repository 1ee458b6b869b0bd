// Per-dispatch overhead of back-to-back launches on one stream: the mean
// launch-to-launch time (events around N launches) against the wall span of
// the blocks themselves (s_memrealtime at block entry and exit, 100 MHz), for
// a 256-block x 512-thread kernel (one block per CU, like the fused forward
// kernel) that computes for a fixed time and writes 0, 2 or 8 MiB, launched
// plainly, with hipExtLaunchKernel, and as a captured hipGraph.
// Build: hipcc --offload-arch=gfx950 -O3 launch_overhead.hip -o launch_overhead
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(512) void k_work(unsigned long long *t, double *out, int nout, int iters, int nt)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    double a = threadIdx.x * 1e-3, b = 1.0;
    for (int k = 0; k < iters; ++k) {
        a = fma(a, 0.999999, 1e-7);
        b = fma(b, 1.000001, -1e-7);
    }
    if (nt >= 3) {
        // blocks of FC = 2^(nt-2) columns x (1024 / FC) rows of the 512 x 512
        // grid; each lane writes one row's FC columns as one vector (a
        // 2^(nt-2) x 8-byte chunk per row: 16, 32, 64 bytes)
        const int FCc = 1 << (nt - 2);
        const unsigned nbk = gridDim.x, full = nbk & ~7u;
        const unsigned lb = blockIdx.x < full ? (blockIdx.x & 7u) * (full >> 3) + (blockIdx.x >> 3) : blockIdx.x;
        const unsigned rows = 1024 / FCc, gy = 512 / rows;
        const unsigned c0 = lb / gy * FCc, r0 = lb % gy * rows;
        for (unsigned r = threadIdx.x; r < rows; r += blockDim.x) {
            double *p = &out[(size_t)(r0 + r) * 512 + c0];
            for (int q = 0; q < FCc; q += 2)
                *(double2 *)(p + q) = make_double2(a + b + q, a - b);
        }
    } else if (nt == 2) {
        // the fused forward kernel's pattern: a 512 x 512 row-major grid, each
        // block 2 columns x 512 rows (16 bytes per row), XCD-aware block order
        const unsigned nbk = gridDim.x, full = nbk & ~7u;
        const unsigned lb = blockIdx.x < full ? (blockIdx.x & 7u) * (full >> 3) + (blockIdx.x >> 3) : blockIdx.x;
        const unsigned ic = lb * 2 + threadIdx.x / 256, r = threadIdx.x % 256;
        for (int i = 0; i < nout; ++i)  // nout = 2: rows r and r + 256 (EPL 2)
            out[(size_t)(i * 256 + r) * 512 + ic] = a + b + i;
    } else {
        const size_t base = (size_t)blockIdx.x * blockDim.x * nout;
        for (int i = 0; i < nout; ++i)
            if (nt) __builtin_nontemporal_store(a + b + i, &out[base + (size_t)i * blockDim.x + threadIdx.x]);
            else out[base + (size_t)i * blockDim.x + threadIdx.x] = a + b + i;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        t[2 * blockIdx.x] = t0;
        t[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

int main()
{
    const int nb = 256, nthr = 512, N = 200;
    unsigned long long *t;
    double *out;
    hipMalloc(&t, 2 * nb * 8);
    hipMalloc(&out, (size_t)nb * nthr * 8 * 8);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<unsigned long long> h(2 * nb);
    for (int iters : {300})
        for (int nout : {0, 2})
            for (int nt : {0, 2, 3, 4, 5, 6})
                for (int mode = 0; mode < 1; ++mode) {
                    if (nout == 0 && nt) continue;
                    auto launch = [&]() {
                        if (mode == 1)
                            hipExtLaunchKernelGGL(k_work, dim3(nb), dim3(nthr), 0, s, nullptr, nullptr, 0u, t, out,
                                                  nout, iters, nt);
                        else
                            hipLaunchKernelGGL(k_work, dim3(nb), dim3(nthr), 0, s, t, out, nout, iters, nt);
                    };
                    hipGraphExec_t ge = nullptr;
                    if (mode == 3) {  // a one-kernel graph, launched N times
                        hipGraph_t g;
                        hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
                        hipLaunchKernelGGL(k_work, dim3(nb), dim3(nthr), 0, s, t, out, nout, iters, nt);
                        hipStreamEndCapture(s, &g);
                        hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
                        hipGraphDestroy(g);
                    }
                    if (mode == 2) {
                        hipGraph_t g;
                        hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
                        for (int i = 0; i < N; ++i) launch();
                        hipStreamEndCapture(s, &g);
                        hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
                        hipGraphDestroy(g);
                    }
                    for (int i = 0; i < 20; ++i) launch();
                    hipStreamSynchronize(s);
                    hipEventRecord(e0, s);
                    if (mode == 2) hipGraphLaunch(ge, s);
                    else if (mode == 3)
                        for (int i = 0; i < N; ++i) hipGraphLaunch(ge, s);
                    else
                        for (int i = 0; i < N; ++i) launch();
                    hipEventRecord(e1, s);
                    hipEventSynchronize(e1);
                    float ms = 0;
                    hipEventElapsedTime(&ms, e0, e1);
                    hipMemcpy(h.data(), t, 2 * nb * 8, hipMemcpyDeviceToHost);
                    unsigned long long lo = ~0ull, hi = 0;
                    double dur = 0;
                    for (int b = 0; b < nb; ++b) {
                        lo = std::min(lo, h[2 * b]);
                        hi = std::max(hi, h[2 * b + 1]);
                        dur += (h[2 * b + 1] - h[2 * b]) * 0.01;
                    }
                    const double per = ms * 1e3 / N, wall = (hi - lo) * 0.01;
                    printf("iters=%5d out=%2d MiB nt=%d %-9s per-launch %6.2f us  block wall %6.2f us  mean block %6.2f us"
                           "  outside blocks %5.2f us\n",
                           iters, nout, nt, mode == 0 ? "plain" : mode == 1 ? "ext" : mode == 2 ? "graph" : "graph1", per, wall, dur / nb,
                           per - wall);
                    if (ge) hipGraphExecDestroy(ge);
                }
    return 0;
}
