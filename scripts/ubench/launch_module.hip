// Per-dispatch overhead of a kernel compiled at run time (hipRTC, loaded with
// hipModuleLoadData, launched with hipExtModuleLaunchKernel -- the engine's
// forward kernels) against the same kernel compiled into the binary, and
// with a large kernel-argument block or dynamic LDS: mean launch-to-launch
// time over N back-to-back launches minus the blocks' wall span.
// Build: hipcc --offload-arch=gfx950 -O3 launch_module.hip -o launch_module -lhiprtc
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>

#define KSRC(NAME, EXTRA)                                                                                      \
    "extern \"C\" __global__ __launch_bounds__(512) void " NAME "(unsigned long long *t, double *out, int iters" \
    EXTRA ")\n{\n"                                                                                              \
    "    extern __shared__ double lds[];\n"                                                                     \
    "    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();\n"                                     \
    "    double a = threadIdx.x * 1e-3, b = 1.0;\n"                                                             \
    "    for (int k = 0; k < iters; ++k) { a = fma(a, 0.999999, 1e-7); b = fma(b, 1.000001, -1e-7); }\n"       \
    "    lds[threadIdx.x] = a;\n"                                                                               \
    "    __syncthreads();\n"                                                                                    \
    "    out[(size_t)blockIdx.x * 512 + threadIdx.x] = lds[511 - threadIdx.x] + b;\n"                           \
    "    if (threadIdx.x == 0) { t[2 * blockIdx.x] = t0; t[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime(); }\n" \
    "}\n"

const char *kSrc = KSRC("k_small", "") KSRC("k_bigargs", ", const double *a1, const double *a2, const double *a3, "
                                                         "double d1, double d2, unsigned u1, unsigned u2, unsigned u3, "
                                                         "const double *a4, const double *a5, unsigned u4, unsigned u5, "
                                                         "double *a6, unsigned u6, const unsigned *a7");

int main()
{
    hiprtcProgram prog;
    hiprtcCreateProgram(&prog, kSrc, "k.hip", 0, nullptr, nullptr);
    const char *opts[] = {"--offload-arch=gfx950", "-O3"};
    if (hiprtcCompileProgram(prog, 2, opts) != HIPRTC_SUCCESS) {
        size_t ls;
        hiprtcGetProgramLogSize(prog, &ls);
        std::string log(ls, 0);
        hiprtcGetProgramLog(prog, &log[0]);
        printf("compile failed: %s\n", log.c_str());
        return 1;
    }
    size_t cs;
    hiprtcGetCodeSize(prog, &cs);
    std::vector<char> code(cs);
    hiprtcGetCode(prog, code.data());
    hipModule_t mod;
    hipModuleLoadData(&mod, code.data());
    hipFunction_t fs, fb;
    hipModuleGetFunction(&fs, mod, "k_small");
    hipModuleGetFunction(&fb, mod, "k_bigargs");
    const int nb = 256, N = 200, iters = 300;
    unsigned long long *t;
    double *out;
    hipMalloc(&t, 2 * nb * 8);
    hipMalloc(&out, (size_t)nb * 512 * 8);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<unsigned long long> h(2 * nb);
    for (int variant = 0; variant < 4; ++variant) {
        const bool big = variant & 1;
        const unsigned dyn = (variant & 2) ? 40 * 1024 : 4096;
        double *p = out;
        unsigned long long *tp = t;
        int it = iters;
        const double *a1 = out;
        double d1 = 1.0;
        unsigned u1 = 1;
        const unsigned *a7 = nullptr;
        double *a6 = out;
        void *args_s[] = {&tp, &p, &it};
        void *args_b[] = {&tp, &p, &it, &a1, &a1, &a1, &d1, &d1, &u1, &u1, &u1, &a1, &a1, &u1, &u1, &a6, &u1, &a7};
        auto launch = [&]() {
            hipExtModuleLaunchKernel(big ? fb : fs, nb * 512, 1, 1, 512, 1, 1, dyn, s, big ? args_b : args_s, nullptr,
                                     nullptr, nullptr, 0);
        };
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
        printf("hipRTC module kernel, %s args, dyn LDS %5u B: per-launch %6.2f us  block wall %6.2f us  outside %5.2f us\n",
               big ? "18" : " 3", dyn, per, wall, per - wall);
    }
    return 0;
}
