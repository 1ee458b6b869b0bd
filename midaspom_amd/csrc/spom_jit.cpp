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
// FNV-1a hash of the generated source, the compile options and the hipRTC
// version; a cached file that is not a gfx950 code object, or that the
// runtime refuses to load (spom_engine.hip jit_load), is rebuilt.  hipRTC
// itself (and the compiler library it brings in) is loaded with dlopen on
// the first cache miss only: a run whose code objects are all cached never
// maps it (the drop-in CLI's start-up, main_MIDASPOM.c:326-332).
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <hip/hiprtc.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <atomic>
#include <mutex>
#include <sstream>
#include <algorithm>
#include <cstdint>
#include <string>
#include <sys/stat.h>
#include <type_traits>
#include <vector>

#include "spom_jit.h"

namespace {

const char *kPrelude = R"SRC(
typedef unsigned int u32;
// log x = k ln2 + log m, x = 2^k m with m in [sqrt(1/2), sqrt(2)): log m =
// 2 atanh(s), s = (m - 1) / (m + 1), |s| <= 0.1716, the odd series to s^21
// (remainder below 2^-62 of the sum).  About 20 FP64 operations and no
// table, a fraction of the library log's cost; within 2 ulp of it
// (tests/test_gpu_parity.py::test_engine_log_accuracy).
__device__ __forceinline__ double mdp_log(double x)
{
    if (!(x > 0.0) || x == __builtin_inf()) return x == 0.0 ? -__builtin_inf() : (x > 0.0 ? x : __builtin_nan(""));
    int k = 0;
    if (x < 0x1p-1022) {  // subnormal: scale into the normal range
        x *= 0x1p54;
        k = -54;
    }
    const unsigned long long ix = (unsigned long long)__double_as_longlong(x);
    k += (int)(ix >> 52) - 1023;
    double m = __longlong_as_double((long long)((ix & 0x000fffffffffffffull) | 0x3ff0000000000000ull));
    if (m > 1.4142135623730951) {
        m *= 0.5;
        ++k;
    }
    const double f = m - 1.0, d = m + 1.0;
    double r = __builtin_amdgcn_rcp(d);  // 1 / d: one Newton step, then a corrected quotient
    r = fma(fma(-d, r, 1.0), r, r);
    double s = f * r;
    s = fma(fma(-d, s, f), r, s);
    const double z = s * s;
    double p = 1.0 / 21.0;
    p = fma(p, z, 1.0 / 19.0);
    p = fma(p, z, 1.0 / 17.0);
    p = fma(p, z, 1.0 / 15.0);
    p = fma(p, z, 1.0 / 13.0);
    p = fma(p, z, 1.0 / 11.0);
    p = fma(p, z, 1.0 / 9.0);
    p = fma(p, z, 1.0 / 7.0);
    p = fma(p, z, 1.0 / 5.0);
    p = fma(p, z, 1.0 / 3.0);
    const double lm = fma(2.0 * s, z * p, 2.0 * s);  // 2 s (1 + z p)
    const double kd = (double)k;
    return fma(kd, 0x1.62e42fefa39efp-1, fma(kd, 0x1.abc9e3b39803fp-56, lm));
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

// The disk cache: MDP_JIT_CACHE, else ~/.cache/midaspom_jit, else (no
// HOME) a per-user /tmp/midaspom_jit-<uid>.  The directory is created 0700
// and used only while it is owned by this user and writable by nobody else
// (cache_dir_private): a code object found there is loaded into the GPU, so
// a directory another user can write to is not a cache.
std::string cache_dir()
{
    if (const char *d = getenv("MDP_JIT_CACHE")) return d;
    if (const char *h = getenv("HOME")) return std::string(h) + "/.cache/midaspom_jit";
    return "/tmp/midaspom_jit-" + std::to_string((long)geteuid());
}

bool cache_dir_private(const std::string &dir)
{
    struct stat st;
    if (lstat(dir.c_str(), &st) != 0 || !S_ISDIR(st.st_mode)) return false;
    return st.st_uid == geteuid() && (st.st_mode & (S_IWGRP | S_IWOTH)) == 0;
}

// create the cache directory (and its parent, e.g. ~/.cache) if missing
void make_cache_dir(const std::string &dir)
{
    const size_t sl = dir.find_last_of('/');
    if (sl != std::string::npos && sl > 0) mkdir(dir.substr(0, sl).c_str(), 0755);
    mkdir(dir.c_str(), 0700);
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
    make_cache_dir(dir);
    if (!cache_dir_private(dir)) return;
    static std::atomic<unsigned> seq{0};  // threads of one process write distinct temporaries
    std::string tmp = path + ".tmp" + std::to_string((long)getpid()) + "." + std::to_string(seq++);
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

namespace {

// The transition P[a][b](e, c) = sum_m Q_ab[m](c) x^(|A|-m) y^m (x = min(e, 1),
// y = 1 - x) is evaluated per point without a weight table, in
// one of two ratio forms chosen per lane:
//   t-form (x >= y): P = x^|A| * H_t,              H_t = sum_m Q[m] t^m,      t = y / x <= 1
//   s-form (x <  y): P = y^|A| * s^(|A|-nX) * H_s, H_s = sum_m Q[m] s^(nX-m), s = x / y <  1
// Both are one Horner chain of nX FMAs over the group's coefficients -- the
// s-form reads them in stored order, the t-form reversed (a second, reversed
// copy of the Q row sits in LDS, so the choice is a per-lane base address).
// Writing B = x (t) or y (s) and g = 1 (t) or s (s):  P = B^|A| g^(|A|-nX) H.
// The factor g^d (d = |A| - nX = |A \ B|, the patches forced extinct) is a
// multiply per transition when d > 0; B^|A| depends only on the source state,
// so it is deferred: every state of a year carries the same pending exponent
// E of B (sources of a year with |A| above the year's minimum are scaled by
// B^(|A| - min) first), applied when E passes kFlushExp and at the end.
// The deferred values are bounded: H <= sum_m Q[m] <= 2^nX <= 2^|A| with both
// ratios <= 1 and B >= 1/2 for e in [0, 1] (B > 1 for e < 0, where nothing
// grows), so a state is at most 2^E np0 times its true value and B^E >= 2^-E.
constexpr uint32_t kFlushExp = 192;

struct Schedule {
    std::vector<uint32_t> amin;          // per year t >= 1: min |A| over the year's sources
    std::vector<std::vector<uint32_t>> diff;  // per year: |A_k| - amin per source k
    std::vector<uint32_t> flush;         // per year: pending exponent applied after it (0: none)
    uint32_t final_exp = 0;              // pending exponent at the end of the program
    uint32_t dp = 0, dg = 0;             // largest source pre-scale and g exponent used
};

Schedule schedule(const MdpJitPlan &pl)
{
    Schedule sc;
    sc.amin.assign(pl.np.size(), 0);
    sc.diff.assign(pl.np.size(), {});
    sc.flush.assign(pl.np.size(), 0);
    uint32_t E = pl.e0;
    size_t u = 0;
    for (size_t t = 1; t < pl.np.size(); ++t) {
        const uint32_t npp = pl.np[t - 1], npc = pl.np[t];
        std::vector<uint32_t> a(npp, 0);
        for (uint32_t l = 0; l < npc; ++l)
            for (uint32_t k = 0; k < npp; ++k) {
                const uint32_t d = pl.udesc[u + (size_t)l * npp + k];
                const uint32_t nX = (d >> 22) & 31u, nA = d >> 27;
                a[k] = nA;  // a use's |A| is its source's
                if (nA > nX) sc.dg = std::max(sc.dg, nA - nX);
            }
        u += (size_t)npp * npc;
        const uint32_t am = *std::min_element(a.begin(), a.end());
        sc.amin[t] = am;
        for (uint32_t k = 0; k < npp; ++k) {
            sc.diff[t].push_back(a[k] - am);
            sc.dp = std::max(sc.dp, a[k] - am);
        }
        E += am;
        if (E >= kFlushExp) {
            sc.flush[t] = E;
            E = 0;
        }
    }
    sc.final_exp = E;
    return sc;
}

// reversed-copy index of every coefficient slot: within each group (offset,
// nX + 1 coefficients) slot off + k holds coefficient off + nX - k; slots of
// no used group map to themselves
std::vector<uint32_t> reversed_index(const std::vector<uint32_t> &udesc, size_t ldq)
{
    std::vector<uint32_t> rev(ldq);
    for (size_t i = 0; i < ldq; ++i) rev[i] = (uint32_t)i;
    for (uint32_t d : udesc) {
        const uint32_t off = d & ((1u << 22) - 1u), nX = (d >> 22) & 31u;
        for (uint32_t k = 0; k <= nX && off + k < ldq; ++k) rev[off + k] = off + nX - k;
    }
    return rev;
}

// B^E (or g^E) for point i as straight-line code: binary powers of `base`
std::string power_expr(const std::string &base, uint32_t E, const std::string &tmp)
{
    if (E == 0) return "1.0";
    std::ostringstream o;
    o << "[&]() { double " << tmp << "_s = " << base << ", " << tmp << "_f = 1.0;";
    bool first = true;
    for (uint32_t b = E; b; b >>= 1) {
        if (!first) o << " " << tmp << "_s *= " << tmp << "_s;";
        if (b & 1u) o << " " << tmp << "_f = " << (first ? tmp + "_s;" : tmp + "_f * " + tmp + "_s;");
        first = false;
    }
    o << " return " << tmp << "_f; }()";
    return o.str();
}

}  // namespace

// The fused kernel's Q-entry sum in the canonical order of spom_engine.hip
// (kQGroup = 8: the items in groups of eight summed left to right, the group
// sums as a pairwise tree over the entry's groups: a binary counter folded
// from its lowest occupied level up).  Every gather is unconditional: slots
// past the entry's count read the zero slot pl[NITEMS] (set in the Pc
// phase), so all loads are in flight at once instead of one branch and wait
// per item.  The groups and the tree then run over the compile-time bound
// (groups of zeros past the entry, a tree padded to a power of two); every
// padded addition is x + (+0.0) = x for the non-negative (or NaN / inf) sums
// here, so the bits are those of the canonical order.  Sets `a`.
std::string qsum_flat_code(uint32_t qml, uint32_t qun)
{
    const uint32_t G = 8, ngm = (qml + G - 1) / G;  // = kQGroup (spom_engine.hip)
    uint32_t ngp = 1;
    while (ngp < ngm) ngp *= 2;
    std::ostringstream o;
    o << "            const u32 cnt_ = qn[k];\n"
         "            double p_[" << qml << "];\n";
    for (uint32_t u = 0; u < qml; ++u) {
        if (u < qun)
            o << "            p_[" << u << "] = pl[qx[k][" << u << "]];\n";
        else
            o << "            { const u32 t_ = Qil[qb[k] + " << u << "u]; p_[" << u << "] = pl[" << u
              << "u < cnt_ ? t_ : (u32)NITEMS]; }\n";
    }
    o << "            (void)cnt_;\n            double g_[" << ngp << "];\n";
    for (uint32_t g = 0; g < ngp; ++g) {
        if (g >= ngm) {
            o << "            g_[" << g << "] = 0.0;\n";
            continue;
        }
        o << "            g_[" << g << "] = p_[" << G * g << "]";
        for (uint32_t u = 1; u < G && G * g + u < qml; ++u) o << " + p_[" << G * g + u << "]";
        o << ";\n";
    }
    for (uint32_t w = ngp; w > 1; w /= 2)
        for (uint32_t i = 0; i < w / 2; ++i)
            o << "            g_[" << i << "] = g_[" << 2 * i << "] + g_[" << 2 * i + 1 << "];\n";
    o << "            const double a = g_[0];\n";
    return o.str();
}

MdpRatioWork mdp_jit_ratio_work(const MdpJitPlan &pl)
{
    MdpRatioWork w;
    if (pl.np.empty()) return w;
    const Schedule sch = schedule(pl);
    // B^E by squaring: floor(log2 E) squarings + popcount(E) - 1 products
    auto powcost = [](uint32_t E) -> double {
        if (E <= 1) return 0.0;
        return (double)(31 - __builtin_clz(E)) + (double)__builtin_popcount(E) - 1.0;
    };
    w.setup_t = 2.0 + (sch.dp > 1 ? sch.dp - 1.0 : 0.0);
    w.setup_s = w.setup_t + (sch.dg > 1 ? sch.dg - 1.0 : 0.0);
    const uint32_t kOffM = (1u << 22) - 1u;
    std::set<uint32_t> groups, gd;
    for (uint32_t d : pl.udesc) {
        const uint32_t off = d & kOffM, nX = (d >> 22) & 31u, nA = d >> 27;
        if (groups.insert(off).second) {
            w.use_s += 2.0 * nX;
            w.use_t += 2.0 * nX;
        }
        if (nA > nX && gd.insert(off | (nA - nX) << 22).second) w.use_s += 1.0;
    }
    double yr = 0.0;
    for (size_t t = 1; t < pl.np.size(); ++t) {
        const double npp = pl.np[t - 1], npc = pl.np[t];
        yr += npc * (2.0 * npp - 1.0);
        for (uint32_t df : sch.diff[t]) yr += df ? 1.0 : 0.0;
        if (sch.flush[t]) yr += npc + powcost(sch.flush[t]);
    }
    w.use_s += yr;
    w.use_t += yr;
    w.final_pt = (double)pl.np.back() + 1.0 + (sch.final_exp ? powcost(sch.final_exp) + 1.0 : 0.0);
    return w;
}

int mdp_jit_default_epl(const std::vector<uint32_t> &) { return 2; }

std::vector<uint32_t> mdp_jit_reversed_index(const std::vector<uint32_t> &udesc, size_t ldq)
{
    return reversed_index(udesc, ldq);
}

uint32_t mdp_jit_end_exp(const MdpJitPlan &plan) { return schedule(plan).final_exp; }

std::string mdp_jit_forward_source(MdpJitPlan &pl)
{
    const Schedule sch = schedule(pl);
    const int EPL = pl.vlds ? (pl.epl == 2 ? 2 : 1) : pl.epl > 0 ? pl.epl : 2;
    pl.epl = EPL;
    const uint32_t np0 = pl.np[0];
    uint32_t npmax = 1;
    for (uint32_t x : pl.np) npmax = x > npmax ? x : npmax;
    std::ostringstream o;
    o << kPrelude;
    const bool gather = !pl.qidx.empty();
    const size_t ldq_local = gather ? ((pl.qidx.size() + 1) & ~(size_t)1) : pl.ldQ;
    o << "#define LOGF(x) " << (pl.fast_log ? "mdp_log(x)" : "log(x)") << "\n";
    o << "#define KBLOCK " << (pl.kblock > 0 ? pl.kblock : 256) << "\n";  // threads per column
    o << "#define EPL " << EPL << "\n#define LDQ " << ldq_local << "\n#define LDQG "
      << (gather ? pl.ldq_row : pl.ldQ) << "\n#define NQG " << pl.qidx.size() << "\n#define NPMAX " << npmax
      << "\n#define DP " << sch.dp << "\n#define DG " << sch.dg << "\n";
    // diagnostic phase stamps: s_memtime (slots 0-3) and s_memrealtime (6, 7)
    auto stamp = [&](int slot) {
        if (!pl.diag) return std::string();
        return std::string("    if (stamps && threadIdx.x == 0) stamps[(size_t)blockIdx.x * 8 + ") +
               std::to_string(slot) + "] = " +
               (slot >= 6 ? "__builtin_amdgcn_s_memrealtime();\n" : "__builtin_amdgcn_s_memtime();\n");
    };
    if (pl.fused)
        o << "#define NJ " << pl.nj << "\n#define NVAR " << pl.nvar << "\n#define NITEMS " << pl.nitems
          << "\n#define NCOEF " << pl.ncoef << "\n#define NQI " << (pl.nqi ? pl.nqi : 1) << "\n#define OFF_IT "
          << pl.off_it << "\n#define OFF_QS " << pl.off_qs << "\n#define OFF_QI " << pl.off_qi << "\n#define OFF_RQ "
          << pl.off_rq << "\n#define OFF_ZC "
          << pl.off_zc << "\n#define OFF_ZS "
          << pl.off_zs << "\n#define KZ " << std::max<uint32_t>(8u, pl.kzmax) << "\n#define ZPAD " << (pl.zpad ? 1 : 0)
          << "\n#define QML "
          << std::max<uint32_t>(1u, pl.qmaxlen) << "\n#define QUN " << std::min<uint32_t>(std::max<uint32_t>(1u, pl.qmaxlen), 16u)
          << "\n#define NSTG "
          << std::max<uint32_t>(1u, (pl.ct_max / 2 + (uint32_t)(pl.kblock * pl.fused_cols * std::max(1, pl.pro)) - 1) /
                                       ((uint32_t)(pl.kblock * pl.fused_cols * std::max(1, pl.pro)))) << "\n";
    // columns per workgroup (KBLOCK threads each; the fused variant).  Two
    // columns per reading workgroup (both Q rows staged, the pair's results
    // stored as one 16-byte store per row through LDS) was measured slower on
    // configs 2 and 3, so the reading variant takes one.
    const int FC = pl.fused ? (pl.fused_cols > 0 ? pl.fused_cols : 1) : 1;
    // target split (vlds): SPL waves per 64 points, wave group `half`
    // accumulating the new states l with l % SPL == half
    const int SPL = pl.vlds && (pl.vsplit == 2 || pl.vsplit == 4) ? pl.vsplit : 1;
    const int PRO = pl.fused && pl.pro > 1 ? pl.pro : 1;
    o << "#define FC " << FC << "\n#define SPL " << SPL << "\n#define NTF (KBLOCK * FC * SPL)\n#define NT (NTF * "
      << PRO << ")\n";
    {   // slot of each coefficient in the reversed copy (see the ratio forms)
        const std::vector<uint32_t> rev = reversed_index(pl.udesc, ldq_local);
        o << "__constant__ const " << (ldq_local <= 65536 ? "unsigned short" : "unsigned int") << " REVQ[" << ldq_local + 2
          << "] = {";
        std::vector<uint32_t> all = rev;
        all.push_back((uint32_t)ldq_local);
        all.push_back((uint32_t)ldq_local + 1);
        for (size_t q = 0; q < all.size(); ++q) o << (q ? (q % 32 ? "," : ",\n") : "") << all[q];
        o << "};\n";
    }
    o << "extern \"C\" __global__ __launch_bounds__(NT) "
      << (pl.wpe > 0 ? "__attribute__((amdgpu_waves_per_eu(" + std::to_string(pl.wpe) + "))) " : std::string())
      << "void mdp_fwd_jit(\n"
         "    const double *__restrict__ Qrow, double prior0, const double *__restrict__ evals, u32 ne, u32 nc,\n"
         "    double *__restrict__ out, u32 ld_out, u32 one, unsigned long long *__restrict__ stamps,\n"
         "    const double *__restrict__ cvals, const double *__restrict__ coltab, u32 ct_len, u32 kmax,\n"
         "    double *__restrict__ vscr, u32 ldv, const u32 *__restrict__ qidx, u32 out_cs,\n"
         "    const u32 *__restrict__ plist, u32 nlist)\n{\n"
         // the Q rows in stored order, then the same rows with every group
         // reversed (read by t-form lanes; see the ratio forms above)
      << "    __shared__ __attribute__((aligned(16))) double Ql[2 * FC * LDQ + 2];\n"
      << stamp(6) << stamp(0) <<
         // XCD-aware order: the dispatcher deals blocks round-robin over the 8
         // XCDs, so consecutive logical blocks (adjacent c columns of the
         // output rows) are given to one XCD and its L2 assembles whole lines
         "    const u32 nb = gridDim.x, full = nb & ~7u;\n"
      << (pl.xcd ? "    const u32 lb = blockIdx.x < full ? (blockIdx.x & 7u) * (full >> 3) + (blockIdx.x >> 3) : blockIdx.x;\n"
                 : "    const u32 lb = blockIdx.x + 0 * full;\n") <<
         // FC columns per workgroup (fused variant): KBLOCK threads each
         "    const u32 half = threadIdx.x / KBLOCK, tid = threadIdx.x % KBLOCK;\n"
         // the lane's place in its column's e block: with several columns per
         // workgroup each column's lanes are rotated by half a block, so the
         // waves a SIMD holds (wave w on SIMD w mod 4) take e rows from both
         // halves -- on a grid with ratio forms split at the block's middle
         // every SIMD then runs one s-form and one t-form wave, not two of one
      << (FC > 1 && SPL == 1 && pl.rot ? "    const u32 tip = (tid + half * (KBLOCK / 2)) % KBLOCK;\n" : "    const u32 tip = tid;\n")
         // (column group, e block): FC columns x KBLOCK*EPL e values per workgroup
      << (pl.efast ? "    const u32 gy = (nlist + KBLOCK * EPL - 1) / (KBLOCK * EPL), ic0 = lb / gy * FC, by = lb % gy;\n"
                   : "    const u32 ncb = (nc + FC - 1) / FC, ic0 = lb % ncb * FC, by = lb / ncb;\n")
      << (SPL > 1 || FC == 1 ? "    const u32 ic = ic0;\n" : "    const u32 ic = ic0 + half;\n")
      << (SPL > 1 ? "    const double *Qh = Ql;\n" : "    const double *Qh = Ql + half * LDQ;\n") <<
         // this lane's points: issued first, their latency hides under the
         // prologue.  One point per lane: e row by * KBLOCK + tid.  Several:
         // list positions pp = by * KBLOCK * EPL + tid * EPL + i, each naming
         // an e row (plist; bit 31: a duplicate that computes but does not
         // store), the host's list putting only points of one ratio form in a
         // lane (set_grid_dev) so that they share their coefficient reads
         "    u32 ie[EPL], pp[EPL];\n    bool st[EPL];\n    double ev[EPL];\n"
         "#pragma unroll\n"
         "    for (int i = 0; i < EPL; ++i) {\n"
      << (EPL == 1 ? "        pp[i] = by * KBLOCK + tip;\n"
                     "        ie[i] = pp[i];\n"
                     "        st[i] = ie[i] < ne;\n"
                   : "        pp[i] = by * (KBLOCK * EPL) + tip * EPL + i;\n"
                     // (no list: the identity, which a sorted grid with an even
                     // number of s-form rows is -- no dependent load then)
                     "        const u32 q_ = pp[i] < nlist ? (plist ? plist[pp[i]] : pp[i]) : 0x80000000u;\n"
                     "        ie[i] = q_ & 0x7fffffffu;\n"
                     "        st[i] = !(q_ >> 31) && ie[i] < ne;\n")
      << "        ev[i] = ie[i] < ne ? evals[ie[i]] : 0.0;\n"
         "    }\n";
    // per point: the ratio form (lane-uniform), the ratio z, the deferred
    // base B, g, and the power tables bp[k] = B^k (source pre-scales, k <= DP)
    // and gp[d] = g^d (d <= DG); then the state vector (emitted before the
    // final prologue barrier)
    std::string wblock;
    {
        std::ostringstream w;
        w << "#pragma unroll\n"
             "    for (int i = 0; i < EPL; ++i) {\n"
             "        const double e = ev[i];\n"
             "        xx[i] = e > 1.0 ? 1.0 : e;\n"
             "        yy[i] = 1.0 - xx[i];\n"
             "    }\n"
             // every point of a lane has one form (the host list), so point 0 decides
             "    const bool tf = xx[0] >= yy[0];\n"
             "    const double *Qp = Qh + (tf ? FC * LDQ : 0);\n"
             "#pragma unroll\n"
             "    for (int i = 0; i < EPL; ++i) {\n"
             "        const double num = tf ? yy[i] : xx[i], den = tf ? xx[i] : yy[i];\n"
             "        zz[i] = num / den;\n"
             "        bb[i] = den;\n"
             "        const double g = tf ? 1.0 : zz[i];\n"
             "        bp[i][0] = 1.0;\n"
             "        gp[i][0] = 1.0;\n"
             "#pragma unroll\n        for (int r = 1; r <= DP; ++r) bp[i][r] = bp[i][r - 1] * den;\n"
             "#pragma unroll\n        for (int r = 1; r <= DG; ++r) gp[i][r] = gp[i][r - 1] * g;\n";
        const char *vdst = pl.vlds ? "Vl[(k * EPL + i) * KBLOCK + tid]" : "v[i][k]";
        // (split: the state k set by wave group k % SPL)
        const char *kloop = SPL > 1 ? "#pragma unroll\n        for (int k = half; k < NPMAX; k += SPL) "
                                    : "#pragma unroll\n        for (int k = 0; k < NPMAX; ++k) ";
        if (pl.first)
            w << kloop << vdst << " = k < " << np0 << " ? 1.0 : 0.0;\n";
        else  // the previous chunk's end vector (ldv covers every lane's list position)
            w << kloop << vdst << " = k < " << np0 << " ? vscr[((size_t)k * nc + ic) * ldv + pp[i]] : 0.0;\n";
        w << "    }\n";
        wblock = w.str();
    }
    o << "    double xx[EPL], yy[EPL], zz[EPL], bb[EPL], bp[EPL][DP + 1], gp[EPL][DG + 1];\n"
         "    double v[EPL][NPMAX];\n    double n[EPL][(NPMAX + SPL - 1) / SPL];\n";
    if (pl.vlds)  // wide years: state k of point i of lane tid at Vl[k][i][tid]
        o << "    __shared__ double Vl[NPMAX * EPL * KBLOCK];\n";
    // the state k of point i, as an expression
    auto vref = [&](uint32_t k) {
        return pl.vlds ? "Vl[(" + std::to_string(k) + " * EPL + i) * KBLOCK + tid]" : "v[i][" + std::to_string(k) + "]";
    };
    if (!pl.fused && !gather) {
        // this column's Q row (k_qrows), in stored order and, through REVQ,
        // with every group reversed: every load in flight before the
        // (unconditional, past the end into a scratch slot) stores, as in stage()
        o << "    {\n"
             "        const double2 *src_ = (const double2 *)(Qrow + (size_t)ic * LDQ);\n"
             "        double2 *dst_ = (double2 *)Ql;\n"
             "        constexpr u32 N2 = LDQ / 2, NK = (N2 + NT - 1) / NT;\n"
             "        double2 t_[NK];\n"
             "        u32 r0_[NK], r1_[NK];\n"
             "#pragma unroll\n"
             "        for (u32 k = 0; k < NK; ++k) {\n"
             "            const u32 i = threadIdx.x + k * NT;\n"
             "            t_[k] = src_[i < N2 ? i : 0];\n"
             "            r0_[k] = i < N2 ? LDQ + REVQ[2 * i] : 2 * LDQ;\n"
             "            r1_[k] = i < N2 ? LDQ + REVQ[2 * i + 1] : 2 * LDQ;\n"
             "        }\n"
             "#pragma unroll\n"
             "        for (u32 k = 0; k < NK; ++k) {\n"
             "            const u32 i = threadIdx.x + k * NT;\n"
             "            dst_[i < N2 ? i : LDQ] = t_[k];\n"
             "            Ql[r0_[k]] = t_[k].x;\n"
             "            Ql[r1_[k]] = t_[k].y;\n"
             "        }\n"
             "    }\n"
          << stamp(1);
    } else if (!pl.fused) {
        // this chunk's coefficients gathered from the column's Q row: every
        // load in flight before the (unconditional) stores, as in stage()
        o << "    {\n"
             "        const double *src_ = Qrow + (size_t)ic * LDQG;\n"
             "        constexpr u32 NK = (NQG + NT - 1) / NT;\n"
             "        u32 x_[NK];\n"
             "        double t_[NK];\n"
             "#pragma unroll\n"
             "        for (u32 k = 0; k < NK; ++k) {\n"
             "            const u32 i = threadIdx.x + k * NT;\n"
             "            x_[k] = qidx[i < NQG ? i : 0];\n"
             "        }\n"
             "#pragma unroll\n"
             "        for (u32 k = 0; k < NK; ++k) t_[k] = src_[x_[k]];\n"
             "#pragma unroll\n"
             "        for (u32 k = 0; k < NK; ++k) {\n"
             "            const u32 i = threadIdx.x + k * NT;\n"
             "            Ql[i < NQG ? i : 2 * LDQ] = t_[k];\n"
             "            Ql[i < NQG ? LDQ + REVQ[i] : 2 * LDQ] = t_[k];\n"
             "        }\n"
             "    }\n"
          << stamp(1);
    } else {
        // the k_qrows phases for this one c value (spom_engine.hip k_qrows):
        // Z per hidden-state row, Pc per item, Q per entry -- all in LDS.
        // The column tables (host-built, 1 KiB-padded: var-column S, items,
        // CSR, then zs as [k/2][row][k%2]) are copied to LDS through registers,
        // all in flight, one barrier.
        o << "    extern __shared__ __attribute__((aligned(16))) double ct[];\n"
             "    __shared__ double Zl[FC * NJ];\n"
             "#define PLS (NITEMS + 1)\n"  // a column's items, then its zero slot (the flat Q sums' padding)
             "    __shared__ double Pl[FC * PLS];\n"
          <<
             "    const uint2 *Itl = (const uint2 *)(ct + OFF_IT);\n"
             "    const u32 *Qsl = (const u32 *)(ct + OFF_QS);\n"
             "    const u32 *Qil = (const u32 *)(ct + OFF_QI);\n"
             // the reversed-copy slots, staged with the tables (REVQ is a
             // global load, issued where used: after the Pc barrier)
             "    const u32 *Rql = (const u32 *)(ct + OFF_RQ);\n"
             "    const double *zcl = ct + OFF_ZC;\n"
             "    const double *Svl = ct;\n"
             "    const double *zl = ct + OFF_ZS;\n"
             "    double cc[FC];\n"
             "#pragma unroll\n"
             "    for (int f = 0; f < FC; ++f) cc[f] = ic0 + f < nc ? cvals[ic0 + f] : 0.0;\n"
             "    {\n"
             "        const double2 *src = (const double2 *)coltab;\n"
             "        double2 *dst = (double2 *)ct;\n"
             "        const u32 n2 = ct_len / 2;\n"
             "        double2 t[NSTG];\n"
             "#pragma unroll\n"
             "        for (int k = 0; k < NSTG; ++k) {\n"
             "            const u32 i = threadIdx.x + k * NT;\n"
             "            t[k] = src[i < n2 ? i : 0];\n"
             "        }\n"
             "#pragma unroll\n"
             "        for (int k = 0; k < NSTG; ++k) {\n"
             "            const u32 i = threadIdx.x + k * NT;\n"
             // unconditional: lanes past the image write a scratch slot, so the
             // loads are not sunk into per-load branches (load, wait, store x NSTG)
             "            dst[i < n2 ? i : n2] = t[k];\n"
             "        }\n"
             "    }\n"
             "    __syncthreads();\n"
          << stamp(4);
        o <<
             // operands of the Pc and Q phases that do not depend on Z, read
             // and combined before the Z phase: per item its Z slot and the
             // product F of its var-column factors (a fixed pairwise tree),
             // per Q entry its item count and first QUN item indices
             "    constexpr int KPC = (FC * NITEMS + NT - 1) / NT;\n"
             "    constexpr int KQ = (FC * LDQ + NT - 1) / NT;\n"
             // item w of pass k: even passes run from the last thread down, so
             // a single pass (config 2: 588 items on 1 024 threads) lands on
             // the waves without Z rows, which then run beside them (round 6:
             // kernel 8.27 -> 8.16 us in the A/B, profiles/r06/cfg2); a wave
             // with no item in a pass skips it (exec-empty branch)
             "    double Fp[KPC];\n"
             "    u32 zi[KPC];\n"
             "#define ITEM_W(k) ((k) * NT + (((k) & 1) ? threadIdx.x : NT - 1 - threadIdx.x))\n"
             "#define ZW(k) ((k) * NT + threadIdx.x)\n#define QW(k) ((k) * NT + threadIdx.x)\n"
"#pragma unroll\n"
             "    for (int k = 0; k < KPC; ++k) {\n"
             "        const u32 w = ITEM_W(k);\n"
             "        Fp[k] = 0.0;\n"
             "        zi[k] = 0u;\n"
             "        if (w >= FC * NITEMS) continue;\n"
             "        const u32 col = w % FC, it = w / FC;\n"
             "        const double c = cc[col];\n"
             "        const uint2 t = Itl[it];\n"
             "        const u32 r = (t.x >> 24) | ((t.y >> 24) << 8), B = t.x & 0xffffffu, j = t.y & 0xffffffu;\n"
             // f_b = j_b ? 1 : B_b ? p_b : 1 - p_b with p_b = min(1, c S): one
             // v_min_f64 for the clamp and j (round 6: the image marks j's
             // columns +inf, so c S is +inf -- or NaN at c = 0, which minNum
             // drops -- and p_b = 1.0; j <= B, so B_b is set there; the
             // compare-and-select form cost 4 more instructions a factor,
             // config 2 8.49 -> 8.32 us, profiles/r06/cfg2), then |n_b - p_b|
             // with n_b = 1.0 where B_b
             // is clear -- the same bits as fma(s, p, n), (s, n) = (1, 0) or
             // (-1, 1) (1 - p rounded once, |0 - p| = p), with the abs moved to
             // the product (k_qrows uses the same fold)
             "        double f[NVAR];\n"
             "        const u32 nB = ~B;\n"
             "        (void)j;\n"
             "#pragma unroll\n"
             "        for (int b = 0; b < NVAR; ++b) {\n"
             "            const u32 bit = NVAR - 1 - b;\n"
             "            const double p = fmin(c * Svl[r * NVAR + b], 1.0);\n"
             "            f[b] = (double)((nB >> bit) & 1u) - p;\n"
             "        }\n"
             "#pragma unroll\n"
             "        for (int b = 0; b < NVAR; b += 2) f[b] = b + 1 < NVAR ? fabs(f[b]) * fabs(f[b + 1]) : fabs(f[b]);\n"
             "#pragma unroll\n"
             "        for (int s = 2; s < NVAR; s *= 2)\n"
             "#pragma unroll\n"
             "            for (int b = 0; b + s < NVAR; b += 2 * s) f[b] *= f[b + s];\n"
             "        Fp[k] = f[0];\n"
             "        zi[k] = col * NJ + r;\n"
             "    }\n"
             "    u32 qb[KQ], qn[KQ], qx[KQ][QUN];\n"
             "#pragma unroll\n"
             "    for (int k = 0; k < KQ; ++k) {\n"
             "        const u32 w = QW(k), q = w % LDQ;\n"
             "        const bool live = w < FC * LDQ && q < NCOEF;\n"
             "        const u32 q0 = live ? Qsl[q] : 0u, q1 = live ? Qsl[q + 1] : 0u;\n"
             "        qb[k] = q0;\n"
             "        qn[k] = q1 - q0;\n"
             // every index load in flight, reading past the entry within the
             // image; slots past the count name the zero slot
             "#pragma unroll\n"
             "        for (int u = 0; u < QUN; ++u) { const u32 t_ = Qil[q0 + u]; qx[k][u] = (u32)u < qn[k] ? t_ : (u32)NITEMS; }\n"
             "    }\n"
             // Z per (column, row): the row's KZ (compile-time bound) values
             // all in flight; rows past kmax contribute fma(-c, 0, 1) = 1 (with
             // ZPAD the image holds those zero rows, so no per-value select)
             "#pragma unroll\n"
             "    for (int k = 0; k < (FC * NJ + NT - 1) / NT; ++k) {\n"
             "        const u32 w = ZW(k);\n"
             "        if (w < FC * NJ) {\n"
             "            const u32 col = w % FC, r = w / FC;\n"
             "            const double c = cc[col];\n"
             "            double sk[KZ];\n"
             "#pragma unroll\n"
             "            for (u32 kk = 0; kk < KZ; kk += 2) {\n"
             "                const double2 t2 = ((const double2 *)zl)[(ZPAD || kk < kmax ? kk : kk % 8u) / 2 * NJ + r];\n"
             "                sk[kk] = t2.x;\n"
             "                sk[kk + 1] = t2.y;\n"
             "            }\n"
             "            double za = 1.0, zb = 1.0, zc = 1.0, zd = 1.0;\n"
             "#pragma unroll\n"
             "            for (u32 kk = 0; kk < KZ; kk += 8) {\n"
             "                const bool in = ZPAD || kk < kmax;\n"
             "#pragma unroll\n"
             "                for (int u = 0; u < 8; ++u) sk[kk + u] = in ? sk[kk + u] : 0.0;\n"
             "                za *= fma(-c, sk[kk + 0], 1.0) * fma(-c, sk[kk + 4], 1.0);\n"
             "                zb *= fma(-c, sk[kk + 1], 1.0) * fma(-c, sk[kk + 5], 1.0);\n"
             "                zc *= fma(-c, sk[kk + 2], 1.0) * fma(-c, sk[kk + 6], 1.0);\n"
             "                zd *= fma(-c, sk[kk + 3], 1.0) * fma(-c, sk[kk + 7], 1.0);\n"
             "            }\n"
             "            double z = (za * zb) * (zc * zd);\n"
             "            if (kmax && !(fma(-c, sk[0], 1.0) > 0.0)) z = 0.0;\n"
             // the row's small columns: exp(-c (P1 + c (P2/2 + ...))), the
             // expression k_zrows evaluates (spom_engine.hip zseries)
             "            {\n"
             "                const double2 *zq = (const double2 *)(zcl + r * 8);\n"
             "                const double2 p01 = zq[0], p23 = zq[1], p45 = zq[2], p67 = zq[3];\n"
             "                double q = p67.y;\n"
             "                q = fma(q, c, p67.x);\n"
             "                q = fma(q, c, p45.y);\n"
             "                q = fma(q, c, p45.x);\n"
             "                q = fma(q, c, p23.y);\n"
             "                q = fma(q, c, p23.x);\n"
             "                q = fma(q, c, p01.y);\n"
             "                q = fma(q, c, p01.x);\n"
             "                z *= exp(-(q * c));\n"
             "            }\n"
             "            Zl[col * NJ + r] = z;\n"
             "        }\n"
             "    }\n"
             "    __syncthreads();\n"
          << stamp(5) <<
             "#pragma unroll\n"
             "    for (int k = 0; k < KPC; ++k) {\n"
             "        const u32 w = ITEM_W(k);\n"
             "        if (w < FC * NITEMS) Pl[(w % FC) * PLS + w / FC] = Zl[zi[k]] * Fp[k];\n"
             "    }\n"
             "    if (threadIdx.x < FC) Pl[threadIdx.x * PLS + NITEMS] = 0.0;\n"
             "    __syncthreads();\n"
          << stamp(1) <<
             // Q entries: the items in CSR (ascending j) order
             "#pragma unroll\n"
             "    for (int k = 0; k < KQ; ++k) {\n"
             "        const u32 w = QW(k);\n"
             "        if (w < FC * LDQ) {\n"
             "            const double *pl = Pl + (w / LDQ) * PLS;\n"
          << qsum_flat_code(std::max<uint32_t>(1u, pl.qmaxlen), std::min<uint32_t>(std::max<uint32_t>(1u, pl.qmaxlen), 16u)) <<
             "            Ql[w] = a;\n"
             "            Ql[FC * LDQ + (w / LDQ) * LDQ + Rql[w % LDQ]] = a;\n"
             "        }\n"
             "    }\n";
    }
    o << wblock;
    o << "    __syncthreads();\n"
      << stamp(2)
      // the prologue's extra threads (PRO > 1) are done: the forward runs on NTF
      << (PRO > 1 ? "    if (threadIdx.x >= NTF) return;\n" : "");
    // H for point i: the Horner chain of a Q group (offset, nX) over the
    // lane's copy of the coefficients (stored order for s-form lanes,
    // reversed for t-form ones).  Transitions of one group (same A & B and B)
    // from sources of different |A| share H and differ only in g^d.
    // Register kernels emit the forward twice (split_forms), once per ratio
    // form behind a lane-uniform branch on tf: the t-form copy reads the
    // reversed coefficients at a fixed base and drops every g^d factor (g = 1
    // there, so the products it leaves out are exact: the same bits), 55 % of
    // config 2's uses; waves of one form run only their copy.  The LDS-state
    // kernels keep one copy (their wave groups already branch per year).
    const bool split_forms = !pl.vlds && pl.split_forms;
    const char *qbase = "Qp";  // the copy being emitted: "Qp", "Qs_" or "Qt_"
    bool gmul = true;          // the copy being emitted multiplies by g^d
    auto hexpr = [&](uint32_t d) {
        const uint32_t off = d & ((1u << 22) - 1u), nX = (d >> 22) & 31u;
        std::string e = std::string(qbase) + "[" + std::to_string(off) + "]";
        for (uint32_t m = 1; m <= nX; ++m)
            e = "fma(" + e + ", zz[i], " + qbase + "[" + std::to_string(off + m) + "])";
        return e;
    };
    auto gfac = [&](uint32_t d) {
        const uint32_t nX = (d >> 22) & 31u, nA = d >> 27;
        return gmul && nA > nX ? " * gp[i][" + std::to_string(nA - nX) + "]" : std::string();
    };
    // Regions are separate basic blocks: each guard value passes through an
    // opaque scalar move, so instruction selection can neither merge regions
    // nor hoist every transition's reads to the top (which spills).
    const int window = pl.window > 0 ? pl.window : 8;
    // (with the states in LDS the guard also clobbers memory, so a state
    // loaded in one region is reloaded in the next rather than held in a
    // register across the year)
    const char *guard = pl.vlds
        ? "    { u32 g_; asm volatile(\"s_mov_b32 %0, %1\" : \"=s\"(g_) : \"s\"(one) : \"memory\"); if (g_) {\n"
        : "    { u32 g_; asm volatile(\"s_mov_b32 %0, %1\" : \"=s\"(g_) : \"s\"(one)); if (g_) {\n";
    const int nslot = pl.slots > 0 ? pl.slots : 0;
    if (nslot > 0) o << "    double pc[EPL][" << nslot << "];\n";
    int since = 0;
    auto fence = [&]() {
        if (++since >= window) {
            o << "    }}\n" << guard;
            since = 0;
        }
    };
    // The order in which each wave group emits the uses: the register
    // kernel in use order (per new state l, ascending k); with the states in
    // LDS, per year source-major (for k: for the group's l), so a region
    // reads each state once and its accumulations are independent chains.
    // Each n[l] still sums ascending k, so the order changes no bits.
    const size_t nu = pl.udesc.size();
    std::vector<std::vector<size_t>> seq(SPL);
    {
        size_t ub = 0;
        for (size_t t = 1; t < pl.np.size(); ++t) {
            const uint32_t npp = pl.np[t - 1], npc = pl.np[t];
            if (!pl.vlds)
                for (size_t j = 0; j < (size_t)npp * npc; ++j) seq[0].push_back(ub + j);
            else
                for (int h = 0; h < SPL; ++h)
                    for (uint32_t k = 0; k < npp; ++k)
                        for (uint32_t l = h; l < npc; l += SPL) seq[h].push_back(ub + (size_t)l * npp + k);
            ub += (size_t)npp * npc;
        }
    }
    // Transition cache: a use whose Q group (same offset = same H) recurs
    // within kHorizon of its wave group's uses keeps its H in one of
    // pl.slots registers; later uses read it.  Slots are evicted
    // farthest-next-use first.  H is computed exactly as inline, so results
    // do not change.  Positions count within the use's wave group.
    const size_t kHorizon = 64;
    const uint32_t kOffM = (1u << 22) - 1u;
    std::vector<int> grp(nu, 0);
    std::vector<size_t> pos(nu, 0), next_pos(nu, SIZE_MAX);
    for (int h = 0; h < SPL; ++h) {
        std::map<uint32_t, size_t> last;
        for (size_t p = seq[h].size(); p-- > 0;) {
            const size_t u = seq[h][p];
            const uint32_t key = pl.udesc[u] & kOffM;
            grp[u] = h;
            pos[u] = p;
            auto it = last.find(key);
            if (it != last.end()) next_pos[u] = it->second;
            last[key] = p;
        }
    }
    // flops per point: the ratio and its power tables, transitions and
    // scalings (below), the prior sum
    double flops = 2.0 + (double)sch.dp + (double)sch.dg + (pl.last ? 2.0 * npmax : 0.0);
    double fcount = 0.0;  // the copy's flops (the first copy's are kept: the s-form, an upper bound)
    std::vector<std::vector<uint32_t>> slot_key(SPL, std::vector<uint32_t>(nslot, 0));
    std::vector<std::vector<size_t>> slot_next(SPL, std::vector<size_t>(nslot, SIZE_MAX));  // SIZE_MAX: free / dead
    // returns the expression for use u (H times its g^d), emitting
    // "pc[i][s] = H;" first when the use fills a slot (inside the caller's
    // per-point loop)
    auto use_expr = [&](size_t u, std::string &pre) -> std::string {
        const uint32_t d = pl.udesc[u], key = d & kOffM;
        const size_t p = pos[u], np_ = next_pos[u];
        std::vector<uint32_t> &skey = slot_key[grp[u]];
        std::vector<size_t> &snext = slot_next[grp[u]];
        const std::string g = gfac(d);
        if (!g.empty()) fcount += 1.0;
        for (int sl = 0; sl < nslot; ++sl)
            if (snext[sl] == p && skey[sl] == key) {
                snext[sl] = np_;
                return "(pc[i][" + std::to_string(sl) + "]" + g + ")";
            }
        fcount += 2.0 * ((d >> 22) & 31u);  // nX FMAs
        const std::string e = hexpr(d);
        if (nslot == 0 || np_ == SIZE_MAX || np_ - p > kHorizon) return "((" + e + ")" + g + ")";
        int best = 0;
        for (int sl = 1; sl < nslot; ++sl)
            if (snext[sl] > snext[best]) best = sl;
        if (snext[best] != SIZE_MAX && snext[best] <= np_) return "((" + e + ")" + g + ")";
        skey[best] = key;
        snext[best] = np_;
        pre = "pc[i][" + std::to_string(best) + "] = " + e + "; ";
        return "(pc[i][" + std::to_string(best) + "]" + g + ")";
    };
    // a year after which the pending exponent is applied: its new states
    // times B^E (one factor per point)
    auto flush_factor = [&](size_t t) { return power_expr("bb[i]", sch.flush[t], "fl"); };
    // source k of year t, scaled by B^(|A_k| - the year's minimum) where that
    // is not 0 (the register kernel scales in place before the year instead)
    auto src = [&](size_t t, uint32_t k) {
        const uint32_t df = sch.diff[t][k];
        return pl.vlds && df ? "(" + vref(k) + " * bp[i][" + std::to_string(df) + "])" : vref(k);
    };
    // one copy of the forward recursion (its own transition-cache state)
    auto emit_body = [&]() {
    for (int h = 0; h < SPL; ++h) {
        std::fill(slot_key[h].begin(), slot_key[h].end(), 0u);
        std::fill(slot_next[h].begin(), slot_next[h].end(), SIZE_MAX);
    }
    fcount = 0.0;
    since = 0;
    o << guard;
    size_t u = 0;
    for (size_t t = 1; t < pl.np.size(); ++t) {
        const uint32_t npp = pl.np[t - 1], npc = pl.np[t];
        if (npp == 1 && npc == 1 && !pl.vlds) {
            std::string pre;
            const std::string e = use_expr(u++, pre);
            o << "    for (int i = 0; i < EPL; ++i) { " << pre << "v[i][0] = v[i][0] * " << e << "; }\n";
            fcount += 1.0;
            if (sch.flush[t]) {
                o << "    for (int i = 0; i < EPL; ++i) v[i][0] *= " << flush_factor(t) << ";\n";
                fcount += 1.0;
            }
            fence();
            continue;
        }
        if (!pl.vlds)
            for (uint32_t k = 0; k < npp; ++k)
                if (sch.diff[t][k]) {
                    o << "    for (int i = 0; i < EPL; ++i) v[i][" << k << "] *= bp[i][" << sch.diff[t][k] << "];\n";
                    fcount += 1.0;
                }
        if (pl.vlds) {
            // states in LDS: wave group h accumulates the new states l = h,
            // h + SPL, ... (a wave-uniform branch when split), source-major;
            // with the split a barrier either side of the write-back (each
            // lane otherwise touches only its own column of Vl)
            const size_t ubase = u;
            const bool split = SPL > 1;
            if (split) o << "    }}\n";
            for (int h = 0; h < SPL; ++h) {
                if (split) {
                    o << (h == 0 ? std::string("    if (half == 0) {\n")
                          : h + 1 < SPL ? "    } else if (half == " + std::to_string(h) + ") {\n"
                                        : std::string("    } else {\n"))
                      << guard;
                    since = 0;
                }
                for (uint32_t k = 0; k < npp; ++k)
                    for (uint32_t l = h; l < npc; l += SPL) {
                        std::string pre;
                        const std::string e = use_expr(ubase + (size_t)l * npp + k, pre);
                        const std::string acc = "n[i][" + std::to_string(l / SPL) + "]";
                        o << "    for (int i = 0; i < EPL; ++i) { " << pre << acc << " = fma(" << src(t, k) << ", " << e
                          << ", " << (k ? acc : std::string("0.0")) << "); }\n";
                        fcount += sch.diff[t][k] ? 1.0 : 0.0;
                        fcount += k ? 2.0 : 1.0;
                        fence();
                    }
                if (split) o << "    }}\n";
            }
            if (split) o << "    }\n    __syncthreads();\n";
            o << "    for (int i = 0; i < EPL; ++i) {\n";
            if (sch.flush[t]) {
                o << "        const double fl_ = " << flush_factor(t) << ";\n";
                fcount += 1.0 + npc;
            }
            for (int h = 0; h < SPL; ++h) {
                if (split)
                    o << (h == 0 ? std::string("        if (half == 0) {\n")
                          : h + 1 < SPL ? "        } else if (half == " + std::to_string(h) + ") {\n"
                                        : std::string("        } else {\n"));
                for (uint32_t l = h; l < npc; l += SPL)
                    o << "            " << vref(l) << " = n[i][" << l / SPL << "]" << (sch.flush[t] ? " * fl_" : "") << ";\n";
            }
            o << (split ? "        }\n    }\n    __syncthreads();\n" : "    }\n");
            if (split) {
                o << guard;
                since = 0;
            }
            u = ubase + (size_t)npp * npc;
            continue;
        }
        // general year: n[.][l] = sum_k v[.][k] P[k][l] in ascending k
        for (uint32_t l = 0; l < npc; ++l)
            for (uint32_t k = 0; k < npp; ++k) {
                std::string pre;
                const std::string e = use_expr(u++, pre);
                o << "    for (int i = 0; i < EPL; ++i) { " << pre << "n[i][" << l << "] = fma(" << vref(k) << ", "
                  << e << ", " << (k ? "n[i][" + std::to_string(l) + "]" : std::string("0.0")) << "); }\n";
                fcount += k ? 2.0 : 1.0;
                fence();
            }
        // states past npc are never read again (a year reads k < npp, and
        // the final sum runs over the last year's states), so they are not
        // zeroed: that was ~5 % of the forward's VALU issue on config 3
        o << "    for (int i = 0; i < EPL; ++i) {\n";
        if (sch.flush[t]) {
            o << "        const double fl_ = " << flush_factor(t) << ";\n";
            fcount += 1.0 + npc;
        }
        for (uint32_t l = 0; l < npc; ++l)
            o << "        " << vref(l) << " = n[i][" << l << "]" << (sch.flush[t] ? " * fl_" : "") << ";\n";
        o << "    }\n";
    }
    o << "    }}\n";
    };
    if (split_forms) {
        // (s-form lanes: the stored coefficients; t-form: the reversed copy)
        o << "    if (!tf) {\n    const double *Qs_ = Qh;\n";
        qbase = "Qs_";
        gmul = true;
        emit_body();
        flops += fcount;
        o << "    } else {\n    const double *Qt_ = Qh + FC * LDQ;\n";
        qbase = "Qt_";
        gmul = false;
        emit_body();
        o << "    }\n";
    } else {
        emit_body();
        flops += fcount;
    }
    // the pending exponent at the end: applied to L (last chunk); a chunk
    // that is not the last hands its states over unscaled (the next one
    // starts from this exponent, plan.e0)
    const std::string fin = power_expr("bb[i]", sch.final_exp, "fe");
    if (sch.final_exp && pl.last) flops += 1.0;
    o << stamp(3) << "#define NPLAST " << pl.np.back() << "\n"
      << (pl.vlds ? "#define VREF(l) Vl[((l) * EPL + i) * KBLOCK + tid]\n" : "#define VREF(l) v[i][l]\n");
    if (pl.last && (pl.hack == 1 || pl.hack == 2))  // measurement only: the result is never stored
        o << "#pragma unroll\n"
             "    for (int i = 0; i < EPL; ++i) {\n"
             "        double L = 0.0;\n"
             "#pragma unroll\n"
             "        for (int l = 0; l < NPLAST; ++l) L += VREF(l) * prior0;\n"
          << (pl.hack == 1 ? "        if (L == 1234.5678 && st[i] && ic < nc) out[(size_t)ie[i] * ld_out + (size_t)ic * out_cs] = log(L);\n"
                           : "        const double lg_ = LOGF(L * " + fin + ");\n"
                             "        if (lg_ == 1234.5678 && st[i] && ic < nc) out[(size_t)ie[i] * ld_out + (size_t)ic * out_cs] = lg_;\n")
          << "    }\n";
    else if (pl.last)
        o << "    if (SPL == 1 || half == 0) {\n"
             "#pragma unroll\n"
             "    for (int i = 0; i < EPL; ++i) {\n"
             "        double L = 0.0;\n"
             "#pragma unroll\n"
             "        for (int l = 0; l < NPLAST; ++l) L += VREF(l) * prior0;\n"
          << (sch.final_exp ? "        L *= " + fin + ";\n" : std::string()) <<
             "        if (st[i] && ic < nc) out[(size_t)ie[i] * ld_out + (size_t)ic * out_cs] = LOGF(L);\n"
             "    }\n"
             "    }\n";
    else  // hand the end vector to the next chunk
        o << "    if (ic < nc) {\n"
             "#pragma unroll\n"
             "        for (int i = 0; i < EPL; ++i) {\n"
             "#pragma unroll\n"
             "            for (int l = 0; l < NPLAST; ++l)\n"
             "                if (SPL == 1 || l % SPL == (int)half) vscr[((size_t)l * nc + ic) * ldv + pp[i]] = VREF(l);\n"
             "        }\n"
             "    }\n";
    o << stamp(7) << "}\n";
    pl.flops_pt = flops;
    o << "// EPL_CHOSEN " << EPL << "\n";
    return o.str();
}

std::string mdp_jit_log_source()
{
    return std::string(kPrelude) +
           "extern \"C\" __global__ void mdp_log_apply(const double *__restrict__ x, double *__restrict__ y, "
           "unsigned long long n)\n{\n"
           "    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;\n"
           "    if (i < n) y[i] = mdp_log(x[i]);\n}\n";
}

namespace {

// hipRTC entry points, resolved from libhiprtc on first use
struct RtcApi {
    bool ok = false;
    std::string err;
    decltype(&hiprtcCreateProgram) create = nullptr;
    decltype(&hiprtcCompileProgram) compile = nullptr;
    decltype(&hiprtcGetProgramLogSize) log_size = nullptr;
    decltype(&hiprtcGetProgramLog) get_log = nullptr;
    decltype(&hiprtcGetCodeSize) code_size = nullptr;
    decltype(&hiprtcGetCode) get_code = nullptr;
    decltype(&hiprtcDestroyProgram) destroy = nullptr;
    decltype(&hiprtcGetErrorString) errstr = nullptr;
};

const RtcApi &rtc()
{
    static RtcApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = nullptr;
        for (const char *name : {"libhiprtc.so.7", "libhiprtc.so"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL))) break;
        if (!h) {
            const char *e = dlerror();
            api.err = std::string("cannot load libhiprtc: ") + (e ? e : "?");
            return;
        }
        bool all = true;
        auto sym = [&](auto &fp, const char *name) {
            fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
            all = all && fp;
        };
        sym(api.create, "hiprtcCreateProgram");
        sym(api.compile, "hiprtcCompileProgram");
        sym(api.log_size, "hiprtcGetProgramLogSize");
        sym(api.get_log, "hiprtcGetProgramLog");
        sym(api.code_size, "hiprtcGetCodeSize");
        sym(api.get_code, "hiprtcGetCode");
        sym(api.destroy, "hiprtcDestroyProgram");
        sym(api.errstr, "hiprtcGetErrorString");
        api.ok = all;
        if (!all) api.err = "libhiprtc lacks an entry point";
    });
    return api;
}

const char *const kJitOpts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
constexpr int kJitNOpts = 3;
constexpr int kJitCacheFormat = 3;  // bump when the cache key or file layout changes

// The compiler's file identity without loading it: the resolved path, size
// and mtime of libhiprtc and libamd_comgr next to the HIP runtime this
// library runs on (located by dladdr), plus LD_LIBRARY_PATH, which can make
// the dlopen in hiprtc_api() find another libhiprtc.  A comgr / hipRTC
// hotfix without a runtime version bump then changes the key.
const std::string &toolchain_identity()
{
    static std::once_flag once;
    static std::string id;
    std::call_once(once, [] {
        Dl_info di{};
        std::string dir;
        if (dladdr((const void *)&hipRuntimeGetVersion, &di) && di.dli_fname) {
            dir = di.dli_fname;
            const size_t sl = dir.rfind('/');
            dir = sl == std::string::npos ? std::string(".") : dir.substr(0, sl);
        }
        for (const char *lib : {"libhiprtc.so.7", "libamd_comgr.so.3"}) {
            const std::string p = dir + "/" + lib;
            struct stat st{};
            char real[4096];
            id += lib;
            if (!dir.empty() && stat(p.c_str(), &st) == 0) {
                id += ' ';
                id += realpath(p.c_str(), real) ? real : p.c_str();
                id += ' ' + std::to_string((long long)st.st_size) + ' ' + std::to_string((long long)st.st_mtime);
            }
            id += ';';
        }
        if (const char *lp = getenv("LD_LIBRARY_PATH")) (id += " ldpath ") += lp;
    });
    return id;
}

// Cache key: the generated source, the compile options, the ROCm release
// (the HIP runtime's version, which hipRTC ships with -- asking hipRTC itself
// would load it on every run), the compiler libraries' file identity and the
// cache format.  A code object built by another toolchain or with other
// options therefore lands under another name.
uint64_t jit_key(const std::string &src)
{
    int rt = 0;
    (void)hipRuntimeGetVersion(&rt);
    std::string k = src;
    k += '\0';
    for (const char *o : kJitOpts) (k += o) += ' ';
    k += "hip " + std::to_string(rt) + " headers " + std::to_string(HIP_VERSION) + " format " +
         std::to_string(kJitCacheFormat) + " tools " + toolchain_identity();
    return fnv1a(k);
}

// Cache files are the code object followed by a 16-byte trailer: "MDPJ", the
// format, and the 64-bit key it was compiled for.  A file whose trailer does
// not name this key (a stale or corrupted file, another format, another
// key's object under this name) is a miss.  The trailer is a staleness and
// corruption check, not an authentication: the key is also the file name.
// What keeps other users' objects out is the directory check
// (cache_dir_private).
constexpr char kTrailerMagic[4] = {'M', 'D', 'P', 'J'};

void add_trailer(std::vector<char> &c, uint64_t key)
{
    const uint32_t fmt = kJitCacheFormat;
    c.insert(c.end(), kTrailerMagic, kTrailerMagic + 4);
    c.insert(c.end(), (const char *)&fmt, (const char *)&fmt + 4);
    c.insert(c.end(), (const char *)&key, (const char *)&key + 8);
}

bool strip_trailer(std::vector<char> &c, uint64_t key)
{
    if (c.size() < 16) return false;
    const char *t = c.data() + c.size() - 16;
    uint32_t fmt;
    uint64_t k;
    memcpy(&fmt, t + 4, 4);
    memcpy(&k, t + 8, 8);
    if (memcmp(t, kTrailerMagic, 4) != 0 || fmt != (uint32_t)kJitCacheFormat || k != key) return false;
    c.resize(c.size() - 16);
    return true;
}

// ... and what precedes it must be an AMDGPU ELF code object for gfx950
// (e_machine EM_AMDGPU = 224, EF_AMDGPU_MACH = 0x04f).
bool plausible_code_object(const std::vector<char> &c)
{
    if (c.size() < 64 || memcmp(c.data(), "\x7f" "ELF", 4) != 0) return false;
    uint16_t machine;
    uint32_t flags;
    memcpy(&machine, c.data() + 18, sizeof machine);
    memcpy(&flags, c.data() + 48, sizeof flags);
    return machine == 224 && (flags & 0xffu) == 0x4fu;
}

}  // namespace

int mdp_jit_compile(const std::string &src, std::vector<char> &code, std::string &log, bool fresh)
{
    const uint64_t key = jit_key(src);
    if (!fresh) {
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
    if (!fresh && !getenv("MDP_JIT_NOCACHE") && cache_dir_private(dir) && read_file(path, code) &&
        strip_trailer(code, key) && plausible_code_object(code)) {
        std::lock_guard<std::mutex> lk(g_mu);
        g_code[key] = code;
        return 0;
    }
    const RtcApi &R = rtc();
    if (!R.ok) {
        log = R.err;
        return -1;
    }
    hiprtcProgram prog;
    if (R.create(&prog, src.c_str(), "mdp_fwd_jit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
        log = "hiprtcCreateProgram failed";
        return -1;
    }
    const hiprtcResult r = R.compile(prog, kJitNOpts, kJitOpts);
    size_t ls = 0;
    R.log_size(prog, &ls);
    if (ls > 1) {
        std::vector<char> lb(ls + 1, 0);
        R.get_log(prog, lb.data());
        log = lb.data();
    }
    if (r != HIPRTC_SUCCESS) {
        R.destroy(&prog);
        if (log.empty()) log = R.errstr(r);
        return -1;
    }
    size_t cs = 0;
    R.code_size(prog, &cs);
    code.resize(cs);
    R.get_code(prog, code.data());
    R.destroy(&prog);
    {
        std::lock_guard<std::mutex> lk(g_mu);
        g_code[key] = code;
    }
    if (!getenv("MDP_JIT_NOCACHE")) {
        std::vector<char> file = code;
        add_trailer(file, key);
        write_file(dir, path, file);
    }
    return 0;
}
