// First-launch cost of a one-kernel fat binary: device count, then the first
// reference to a static kernel (hipFuncGetAttributes loads the code object),
// then a launch.  Compared with and without a warm comgr cache by
// scripts/jitcache_probe.py.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_tiny(double *p) { p[threadIdx.x] = threadIdx.x; }

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main()
{
    int n = 0;
    const double t0 = now();
    (void)hipGetDeviceCount(&n);
    const double t1 = now();
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, (const void *)k_tiny);
    const double t2 = now();
    double *p = nullptr;
    (void)hipMalloc(&p, 64 * sizeof(double));
    hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, 0, p);
    (void)hipDeviceSynchronize();
    const double t3 = now();
    fprintf(stderr, "tiny_launch: count %.3f first-kernel-ref %.3f launch %.3f\n", t1 - t0, t2 - t1, t3 - t2);
    (void)hipFree(p);
    return 0;
}
