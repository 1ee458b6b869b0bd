// Block start spread of a 256-block launch (one block per CU) against block
// size, dynamic LDS and VGPR footprint: s_memrealtime (100 MHz) at entry.
// Build: hipcc --offload-arch=gfx950 -O3 dispatch_ramp.hip -o dispatch_ramp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

template <int NREG>
__global__ __launch_bounds__(512) void k_ramp(unsigned long long *t, double *sink, int iters)
{
    extern __shared__ double lds[];
    if (threadIdx.x == 0) t[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    double acc[NREG];
#pragma unroll
    for (int i = 0; i < NREG; ++i) acc[i] = threadIdx.x + i;
    for (int k = 0; k < iters; ++k)
#pragma unroll
        for (int i = 0; i < NREG; ++i) acc[i] = fma(acc[i], 1.0000001, 0.5);
    double s = 0;
#pragma unroll
    for (int i = 0; i < NREG; ++i) s += acc[i];
    lds[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) sink[blockIdx.x] = lds[5];
}

template <int NREG>
void run(int threads, size_t ldsb, const char *tag)
{
    unsigned long long *t;
    double *sink;
    hipMalloc(&t, 256 * 8);
    hipMalloc(&sink, 256 * 8);
    std::vector<unsigned long long> h(256);
    double spread = 0;
    for (int rep = 0; rep < 6; ++rep) {
        hipLaunchKernelGGL(k_ramp<NREG>, dim3(256), dim3(threads), ldsb, 0, t, sink, 2000);
        hipDeviceSynchronize();
        hipMemcpy(h.data(), t, 256 * 8, hipMemcpyDeviceToHost);
        auto mm = std::minmax_element(h.begin(), h.end());
        if (rep) spread += (*mm.second - *mm.first) * 0.01;  // us
    }
    // back to back: 20 launches, no synchronisation between them; the
    // stamps are the last launch's
    double spread2 = 0;
    for (int rep = 0; rep < 5; ++rep) {
        for (int i = 0; i < 20; ++i)
            hipLaunchKernelGGL(k_ramp<NREG>, dim3(256), dim3(threads), ldsb, 0, t, sink, 2000);
        hipDeviceSynchronize();
        hipMemcpy(h.data(), t, 256 * 8, hipMemcpyDeviceToHost);
        auto mm = std::minmax_element(h.begin(), h.end());
        spread2 += (*mm.second - *mm.first) * 0.01;
    }
    printf("%-34s threads=%4d lds=%6zu  start spread after idle %.2f us, back to back %.2f us\n", tag, threads,
           ldsb, spread / 5, spread2 / 5);
    hipFree(t);
    hipFree(sink);
}

int main()
{
    hipFuncSetAttribute((const void *)k_ramp<80>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    hipFuncSetAttribute((const void *)k_ramp<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    run<8>(256, 8192, "small regs, 256 thr");
    run<8>(512, 8192, "small regs, 512 thr");
    run<8>(512, 40960, "small regs, 512 thr, 40 KB LDS");
    run<80>(512, 8192, "~170 VGPRs, 512 thr");
    run<80>(512, 40960, "~170 VGPRs, 512 thr, 40 KB LDS");

    return 0;
}
