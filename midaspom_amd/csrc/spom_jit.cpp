// midaspom_amd/csrc/spom_jit.cpp -- problem-specialised forward kernel.
//
// The forward recursion of the reference (main_MIDASPOM.c:368-392) has a
// control structure fixed by the observation file alone: the number of
// possible states in each year.  At engine creation we emit it as
// straight-line HIP source -- one block per year, every transition's
// coefficient block at a compile-time LDS offset -- and compile it for gfx950
// with hipRTC.  With no data-dependent branches left, the compiler can issue
// the LDS reads of later transitions under the arithmetic of earlier ones;
// the runtime-shape kernels in spom_engine.hip serialise on every general
// year instead.  Code objects are cached in memory and on disk, keyed by the
// FNV-1a hash of the generated source.
#include <hip/hiprtc.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <sys/stat.h>
#include <vector>

#include "spom_jit.h"

namespace {

const char *kPrelude = R"SRC(
typedef unsigned int u32;
#define KBLOCK 256
template <int RS>
__device__ __forceinline__ double tdot(const double *p, const double (&w)[RS])
{
    // coefficient block at a 16-byte aligned LDS address: ds_read_b128 pairs
    double c[RS];
    const double2 *p2 = (const double2 *)p;
#pragma unroll
    for (int r = 0; r + 1 < RS; r += 2) {
        const double2 q = p2[r / 2];
        c[r] = q.x;
        c[r + 1] = q.y;
    }
    if (RS & 1) c[RS - 1] = p[RS - 1];
    double a0 = 0.0, a1 = 0.0;
#pragma unroll
    for (int r = 0; r + 1 < RS; r += 2) {
        a0 = fma(c[r], w[r], a0);
        a1 = fma(c[r + 1], w[r + 1], a1);
    }
    if (RS & 1) a0 = fma(c[RS - 1], w[RS - 1], a0);
    return a0 + a1;
}
)SRC";

uint64_t fnv1a(const std::string &s)
{
    uint64_t h = 1469598103934665603ull;
    for (unsigned char c : s) {
        h ^= c;
        h *= 1099511628211ull;
    }
    return h;
}

std::string cache_dir()
{
    if (const char *d = getenv("MDP_JIT_CACHE")) return d;
    if (const char *h = getenv("HOME")) {
        std::string p = std::string(h) + "/.cache/midaspom_jit";
        return p;
    }
    return "/tmp/midaspom_jit";
}

bool read_file(const std::string &path, std::vector<char> &out)
{
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) return false;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    rewind(f);
    if (n <= 0) {
        fclose(f);
        return false;
    }
    out.resize((size_t)n);
    bool ok = fread(out.data(), 1, (size_t)n, f) == (size_t)n;
    fclose(f);
    return ok;
}

void write_file(const std::string &dir, const std::string &path, const std::vector<char> &data)
{
    mkdir(dir.c_str(), 0755);  // one level is enough for the default layouts
    std::string parent = dir.substr(0, dir.find_last_of('/'));
    mkdir(parent.c_str(), 0755);
    mkdir(dir.c_str(), 0755);
    std::string tmp = path + ".tmp" + std::to_string((long)getpid());
    FILE *f = fopen(tmp.c_str(), "wb");
    if (!f) return;
    const bool ok = fwrite(data.data(), 1, data.size(), f) == data.size();
    fclose(f);
    if (ok) rename(tmp.c_str(), path.c_str());
    else remove(tmp.c_str());
}

std::mutex g_mu;
std::map<uint64_t, std::vector<char>> g_code;  // in-process code-object cache

}  // namespace

std::string mdp_jit_forward_source(const MdpJitPlan &pl)
{
    const int RS = (int)pl.deg + 1;
    const int RSP = ((int)pl.deg + 2) & ~1;
    const int EPL = pl.epl;
    const uint32_t np0 = pl.np[0];
    uint32_t npmax = 1;
    for (uint32_t x : pl.np) npmax = x > npmax ? x : npmax;
    std::ostringstream o;
    o << kPrelude;
    o << "#define RS " << RS << "\n#define RSP " << RSP << "\n#define EPL " << EPL << "\n#define LDR "
      << pl.ldR << "\n#define NPMAX " << npmax << "\n";
    o << "extern \"C\" __global__ __launch_bounds__(KBLOCK) void mdp_fwd_jit(\n"
         "    const double *__restrict__ R, double prior0, const double *__restrict__ evals, u32 ne,\n"
         "    double *__restrict__ out, u32 ld_out, u32 one)\n{\n"
         "    __shared__ __attribute__((aligned(16))) double Rl[LDR];\n"
         "    const u32 ic = blockIdx.x;\n"
         "    {\n"
         "        const double2 *src = (const double2 *)(R + (size_t)ic * LDR);\n"
         "        double2 *dst = (double2 *)Rl;\n"
         "        for (u32 i0 = threadIdx.x; i0 < LDR / 2; i0 += 4 * KBLOCK) {\n"
         "            // four loads in flight per lane; clamped indexes keep them unconditional\n"
         "            const u32 i1 = i0 + KBLOCK, i2 = i0 + 2 * KBLOCK, i3 = i0 + 3 * KBLOCK;\n"
         "            const double2 t0 = src[i0];\n"
         "            const double2 t1 = src[i1 < LDR / 2 ? i1 : i0];\n"
         "            const double2 t2 = src[i2 < LDR / 2 ? i2 : i0];\n"
         "            const double2 t3 = src[i3 < LDR / 2 ? i3 : i0];\n"
         "            dst[i0] = t0;\n"
         "            if (i1 < LDR / 2) dst[i1] = t1;\n"
         "            if (i2 < LDR / 2) dst[i2] = t2;\n"
         "            if (i3 < LDR / 2) dst[i3] = t3;\n"
         "        }\n"
         "    }\n"
         "    u32 ie[EPL];\n    double W[EPL][RS];\n    double v[EPL][NPMAX];\n    double n[EPL][NPMAX];\n"
         "#pragma unroll\n"
         "    for (int i = 0; i < EPL; ++i) {\n"
         "        ie[i] = blockIdx.y * (KBLOCK * EPL) + i * KBLOCK + threadIdx.x;\n"
         "        const double e = ie[i] < ne ? evals[ie[i]] : 0.0;\n"
         "        const double x = e > 1.0 ? 1.0 : e;\n"
         "        const double y = 1.0 - x;\n"
         "        double yp[RS];\n        yp[0] = 1.0;\n"
         "#pragma unroll\n        for (int r = 1; r < RS; ++r) yp[r] = yp[r - 1] * y;\n"
         "        double xp = 1.0;\n"
         "#pragma unroll\n        for (int r = RS - 1; r >= 0; --r) { W[i][r] = xp * yp[r]; xp *= x; }\n"
         "#pragma unroll\n        for (int k = 0; k < NPMAX; ++k) v[i][k] = k < "
      << np0 << " ? 1.0 : 0.0;\n"
                "    }\n"
                "    __syncthreads();\n";
    // one block per year transition, uses in (l, k) order as the plan's R.
    // A sched_barrier every `window` transitions bounds how far the scheduler
    // hoists LDS reads (unbounded, straight-line code spills hundreds of VGPRs).
    const int window = pl.window > 0 ? pl.window : 4;
    size_t u = 0, since = 0;
    // Regions are separate basic blocks (an opaque always-true kernel
    // argument guards each), which instruction selection cannot merge.
    // each guard value passes through an opaque scalar move, so no two
    // regions can be proven equivalent and merged
    const char *guard = "    { u32 g_; asm volatile(\"s_mov_b32 %0, %1\" : \"=s\"(g_) : \"s\"(one)); if (g_) {\n";
    o << guard;
    auto fence = [&](size_t uses) {
        since += uses;
        if ((int)since >= window) {
            o << "    }}\n" << guard;
            since = 0;
        }
    };
    for (size_t t = 1; t < pl.np.size(); ++t) {
        const uint32_t npp = pl.np[t - 1], npc = pl.np[t];
        if (npp == 1 && npc == 1) {
            o << "    for (int i = 0; i < EPL; ++i) v[i][0] = v[i][0] * tdot<RS>(Rl + " << u * RSP
              << ", W[i]);\n";
            ++u;
            fence(1);
            continue;
        }
        // general year: n[.][l] = sum_k v[.][k] P[k][l] (ascending k), one
        // statement per transition so a region boundary may fall inside
        for (uint32_t l = 0; l < npc; ++l)
            for (uint32_t k = 0; k < npp; ++k, ++u) {
                o << "    for (int i = 0; i < EPL; ++i) n[i][" << l << "] = fma(v[i][" << k
                  << "], tdot<RS>(Rl + " << u * RSP << ", W[i]), " << (k ? "n[i][" + std::to_string(l) + "]" : std::string("0.0"))
                  << ");\n";
                fence(1);
            }
        o << "    for (int i = 0; i < EPL; ++i) {\n";
        for (uint32_t l = 0; l < npmax; ++l) {
            if (l < npc) o << "        v[i][" << l << "] = n[i][" << l << "];\n";
            else o << "        v[i][" << l << "] = 0.0;\n";
        }
        o << "    }\n";
    }
    o << "    }}\n";
    o << "#pragma unroll\n"
         "    for (int i = 0; i < EPL; ++i) {\n"
         "        double L = 0.0;\n"
         "#pragma unroll\n"
         "        for (int l = 0; l < NPMAX; ++l) L += v[i][l] * prior0;\n"
         "        if (ie[i] < ne) out[(size_t)ie[i] * ld_out + ic] = log(L);\n"
         "    }\n}\n";
    return o.str();
}

int mdp_jit_compile(const std::string &src, std::vector<char> &code, std::string &log)
{
    const uint64_t key = fnv1a(src);
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_code.find(key);
        if (it != g_code.end()) {
            code = it->second;
            return 0;
        }
    }
    char name[64];
    snprintf(name, sizeof name, "fwd_%016llx.co", (unsigned long long)key);
    const std::string dir = cache_dir();
    const std::string path = dir + "/" + name;
    if (!getenv("MDP_JIT_NOCACHE") && read_file(path, code)) {
        std::lock_guard<std::mutex> lk(g_mu);
        g_code[key] = code;
        return 0;
    }
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "mdp_fwd_jit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
        log = "hiprtcCreateProgram failed";
        return -1;
    }
    const char *opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
    const hiprtcResult r = hiprtcCompileProgram(prog, 3, opts);
    size_t ls = 0;
    hiprtcGetProgramLogSize(prog, &ls);
    if (ls > 1) {
        std::vector<char> lb(ls + 1, 0);
        hiprtcGetProgramLog(prog, lb.data());
        log = lb.data();
    }
    if (r != HIPRTC_SUCCESS) {
        hiprtcDestroyProgram(&prog);
        if (log.empty()) log = hiprtcGetErrorString(r);
        return -1;
    }
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    code.resize(cs);
    hiprtcGetCode(prog, code.data());
    hiprtcDestroyProgram(&prog);
    {
        std::lock_guard<std::mutex> lk(g_mu);
        g_code[key] = code;
    }
    if (!getenv("MDP_JIT_NOCACHE")) write_file(dir, path, code);
    return 0;
}
