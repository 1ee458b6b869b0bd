// midaspom_amd/csrc/spom_scenario.hip -- MI355X engine for the reference's two
// scenario likelihoods:
//   in-situ die-off  /root/reference/sources/main_MIDASPOM_dieoff.c:304-351
//   habitat loss     /root/reference/sources/main_MIDASPOM_loss.c:341-386
//
// Both evaluate, for every grid point, L = sum_i sum_s [PK^ts P^tdis]_{i,s}
// prior_s over the full 2^n state space of the FIRST survey row (s its
// observed states), with
//   P  = Pe(e) Pc(c)                    (after the event; K = 1, no source)
//   PK = Pe(e/K) Pc(c, K)   [die-off]   or   Pe(e) Pc_source(c, K, dsrc)  [loss].
// The reference forms the 2^n x 2^n matrices and their powers (matpow: 256^3
// dgemms for n = 8).  Here the powers are never formed:
//   v = P^tdis w,  y = PK^ts v,  L = 1^T y          (column propagation)
// and every operator application factorises:
//   * Pe is a tensor product over patches (per patch: [[1,0],[E,1-E]]), so
//     Pe t is n in-place passes of 2^(n-1) pair updates;
//   * Pc[j][b] (j <= b, 3^n entries) is tabulated once per (c, K, dsrc) in LDS
//     in the reference's factor order, and (Pc y)[j] = sum_{b >= j} Pc[j][b] y[b].
//
// Workgroup = one (c, K, dsrc) point x kE e values; lanes run over e, so the
// Pc table entries are LDS broadcasts and the state vectors y[state][e] are
// read at consecutive addresses.  j rows are processed in popcount groups so
// every lane of a wave does the same amount of work.  k_scn_v computes v per
// (c, e) once (shared by every K); k_scn_lik the rest.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "mdp_internal.h"

namespace {

constexpr int kScnBlock = 256;
constexpr int kE = 16;                 // e values per workgroup (lanes mod 16)
constexpr int kJPar = kScnBlock / kE;  // j rows in flight per workgroup
constexpr uint32_t kMaxN = 8;          // 3^8 Pc entries = 52 KB of LDS

#define SCN_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return mdp_set_error(MDP_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                                 __FILE__, __LINE__);                                        \
    } while (0)

struct ScnArgs {
    uint32_t n, ns, nterm;   // patches, 2^n states, 3^n Pc entries
    int ts, tdis, loss;
    uint32_t ne, nc, nK, nd;
    uint32_t njord;          // row schedule length (kJPar groups x rows, padded with ns)
};

// (Pc y)[j] = sum over supersets b of j, ascending (b = j | sub, sub over
// the submasks of `free` by sub <- (sub - free) & free), of Pc[j][b] y[b].
// Four independent partial sums (terms r mod 4) keep four LDS reads in
// flight per lane; the sum is ((a0 + a1) + (a2 + a3)).
__device__ __forceinline__ double apply_row(const double *__restrict__ tt, const double *__restrict__ y, uint32_t j,
                                            uint32_t free, uint32_t f, uint32_t le)
{
    if (f < 2) {
        double acc = tt[0] * y[j * kE + le];
        if (f == 1) acc += tt[1] * y[(j | free) * kE + le];
        return acc;
    }
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    uint32_t sub = 0;
    for (uint32_t r = 0; r < (1u << f); r += 4) {
        const uint32_t s1 = (sub - free) & free, s2 = (s1 - free) & free, s3 = (s2 - free) & free;
        const double t0 = tt[r], t1 = tt[r + 1], t2 = tt[r + 2], t3 = tt[r + 3];
        const double y0 = y[(j | sub) * kE + le], y1 = y[(j | s1) * kE + le];
        const double y2 = y[(j | s2) * kE + le], y3 = y[(j | s3) * kE + le];
        a0 += t0 * y0;
        a1 += t1 * y1;
        a2 += t2 * y2;
        a3 += t3 * y3;
        sub = (s3 - free) & free;
    }
    return (a0 + a1) + (a2 + a3);
}

// Pc table of one (c, K, source) point into LDS:  T[toff[j] + r] for the r-th
// superset b of j (ascending b) = prod over k not in j, ascending, of
// (b_k ? pC_jk : 1 - pC_jk);  dieoff.c:66-83 pC = (c*S)*K,  loss.c:86-105
// pC = c*(S + src_k*Ks).  Factors 1.0 of occupied patches are skipped (exact).
__device__ void build_table(double *T, double *pc, const double *__restrict__ S, const uint32_t *__restrict__ toff,
                            const uint32_t n, const uint32_t ns, double c, double K, const double *src, double Ks)
{
    // pC for every (j, k), k not in j
    for (uint32_t i = threadIdx.x; i < ns * n; i += kScnBlock) {
        const uint32_t j = i / n, k = i - j * n;
        double v = 0.0;
        if (!((j >> (n - 1 - k)) & 1u)) {
            if (src) v = c * (S[i] + src[k] * Ks);
            else v = c * S[i] * K;
            v = v > 1.0 ? 1.0 : v;
        }
        pc[i] = v;
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x / 16; j < ns; j += kScnBlock / 16) {
        const uint32_t free = ~j & (ns - 1), f = __popc(free);
        for (uint32_t r = threadIdx.x % 16; r < (1u << f); r += 16) {
            uint32_t b = j, xs = free;  // deposit r into the free bits (ascending b)
            for (uint32_t t = 0; t < f; ++t) {
                const uint32_t low = xs & (0u - xs);
                if ((r >> t) & 1u) b |= low;
                xs ^= low;
            }
            double res = 1.0;
            for (uint32_t k = 0; k < n; ++k) {
                const uint32_t bit = 1u << (n - 1 - k);
                if (j & bit) continue;
                const double p = pc[j * n + k];
                res *= (b & bit) ? p : 1.0 - p;
            }
            T[toff[j] + r] = res;
        }
    }
    __syncthreads();
}

// v = P^tdis w for kE e values of one c.  V[c][e-chunk][state][kE].
__global__ __launch_bounds__(kScnBlock) void k_scn_v(ScnArgs a, const double *__restrict__ S,
                                                       const uint32_t *__restrict__ toff,
                                                       const uint32_t *__restrict__ jord,
                                                       const double *__restrict__ w, const double *__restrict__ ev,
                                                       const double *__restrict__ cv, double *__restrict__ V)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double *T = lds, *y = T + a.nterm, *yb = y + a.ns * kE, *pc = yb;  // pc aliases yb before use
    const uint32_t nchunk = (a.ne + kE - 1) / kE;
    const uint32_t ic = blockIdx.x / nchunk, chunk = blockIdx.x % nchunk, e0 = chunk * kE;
    build_table(T, pc, S, toff, a.n, a.ns, cv[ic], 1.0, nullptr, 0.0);
    for (uint32_t i = threadIdx.x; i < a.ns * kE; i += kScnBlock) y[i] = w[i / kE];
    __syncthreads();
    const uint32_t le = threadIdx.x % kE;
    // the extinction probability of every e of the workgroup, for the Pe passes
    __shared__ double Es[kE];
    if (threadIdx.x < kE) {
        double x = e0 + threadIdx.x < a.ne ? ev[e0 + threadIdx.x] : 0.0;
        Es[threadIdx.x] = x > 1.0 ? 1.0 : x;  // loss.c:57-58 (dieoff with K = 1)
    }
    __syncthreads();
    for (int t = 0; t < a.tdis; ++t) {
        // Pc then Pe with per-e E
        const uint32_t jq = threadIdx.x / kE;
        for (uint32_t g = jq; g < a.njord; g += kJPar) {
            const uint32_t j = jord[g];
            if (j >= a.ns) continue;  // padding of the row schedule
            const uint32_t free = ~j & (a.ns - 1), f = __popc(free);
            const double *tt = T + toff[j];
            yb[j * kE + le] = apply_row(tt, y, j, free, f, le);
        }
        __syncthreads();
        for (uint32_t k = 0; k < a.n; ++k) {
            const uint32_t m = 1u << (a.n - 1 - k);
            for (uint32_t i = threadIdx.x; i < (a.ns / 2) * kE; i += kScnBlock) {
                const uint32_t pe = i % kE, pr = i / kE;
                const uint32_t lo = ((pr & ~(m - 1)) << 1) | (pr & (m - 1)), hi = lo | m;
                const double E = Es[pe];
                yb[hi * kE + pe] = E * yb[lo * kE + pe] + (1.0 - E) * yb[hi * kE + pe];
            }
            __syncthreads();
        }
        for (uint32_t i = threadIdx.x; i < a.ns * kE; i += kScnBlock) y[i] = yb[i];
        __syncthreads();
    }
    double *dst = V + ((size_t)ic * nchunk + chunk) * a.ns * kE;
    for (uint32_t i = threadIdx.x; i < a.ns * kE; i += kScnBlock) dst[i] = y[i];
}

// L[e][c][K][d] = 1^T PK^ts v(e, c) for kE e values of one (c, K, d) point.
__global__ __launch_bounds__(kScnBlock) void k_scn_lik(ScnArgs a, const double *__restrict__ S,
                                                         const uint32_t *__restrict__ toff,
                                                         const uint32_t *__restrict__ jord,
                                                         const double *__restrict__ V, const double *__restrict__ ev,
                                                         const double *__restrict__ cv, const double *__restrict__ Kv,
                                                         const double *__restrict__ srcv, double *__restrict__ out)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double *T = lds, *y = T + a.nterm, *yb = y + a.ns * kE, *pc = yb;
    __shared__ double Es[kE];
    const uint32_t nchunk = (a.ne + kE - 1) / kE;
    const uint32_t pt = blockIdx.x / nchunk, chunk = blockIdx.x % nchunk, e0 = chunk * kE;  // (c, K, d) point
    const uint32_t id = pt % a.nd, iK = (pt / a.nd) % a.nK, ic = pt / (a.nd * a.nK);
    const double c = cv[ic], K = Kv[iK];
    build_table(T, pc, S, toff, a.n, a.ns, c, a.loss ? 1.0 : K, a.loss ? srcv + (size_t)id * a.n : nullptr, K);
    const double *vsrc = V + ((size_t)ic * nchunk + chunk) * a.ns * kE;
    for (uint32_t i = threadIdx.x; i < a.ns * kE; i += kScnBlock) y[i] = vsrc[i];
    if (threadIdx.x < kE) {
        const double x = e0 + threadIdx.x < a.ne ? ev[e0 + threadIdx.x] : 0.0;
        double E = a.loss ? x : x / K;  // dieoff.c:56-57 E = e/K; loss.c:57 E = e
        Es[threadIdx.x] = E > 1.0 ? 1.0 : E;
    }
    __syncthreads();
    const uint32_t le = threadIdx.x % kE, jq = threadIdx.x / kE;
    for (int t = 0; t < a.ts; ++t) {
        for (uint32_t g = jq; g < a.njord; g += kJPar) {
            const uint32_t j = jord[g];
            if (j >= a.ns) continue;  // padding of the row schedule
            const uint32_t free = ~j & (a.ns - 1), f = __popc(free);
            const double *tt = T + toff[j];
            yb[j * kE + le] = apply_row(tt, y, j, free, f, le);
        }
        __syncthreads();
        for (uint32_t k = 0; k < a.n; ++k) {
            const uint32_t m = 1u << (a.n - 1 - k);
            for (uint32_t i = threadIdx.x; i < (a.ns / 2) * kE; i += kScnBlock) {
                const uint32_t pe = i % kE, pr = i / kE;
                const uint32_t lo = ((pr & ~(m - 1)) << 1) | (pr & (m - 1)), hi = lo | m;
                const double E = Es[pe];
                yb[hi * kE + pe] = E * yb[lo * kE + pe] + (1.0 - E) * yb[hi * kE + pe];
            }
            __syncthreads();
        }
        for (uint32_t i = threadIdx.x; i < a.ns * kE; i += kScnBlock) y[i] = yb[i];
        __syncthreads();
    }
    // L = sum over states, ascending, per e
    if (threadIdx.x < kE) {
        double L = 0.0;
        for (uint32_t s = 0; s < a.ns; ++s) L += y[s * kE + threadIdx.x];
        const uint32_t ie = e0 + threadIdx.x;
        if (ie < a.ne) out[(((size_t)ie * a.nc + ic) * a.nK + iK) * a.nd + id] = L;
    }
}

template <typename T>
int dev_up(T **p, const std::vector<T> &h)
{
    *p = nullptr;
    SCN_TRY(hipMalloc((void **)p, std::max<size_t>(1, h.size()) * sizeof(T)));
    if (!h.empty()) SCN_TRY(hipMemcpy(*p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return MDP_OK;
}

}  // namespace

struct mdp_scenario {
    uint32_t n = 0, ns = 0, nterm = 0;
    int kind = 0;  // 0 die-off, 1 habitat loss
    double m = 400.0, d = 200.0;
    int device = 0;
    std::vector<double> S, w;
    std::vector<uint32_t> toff, jord;
    double *dS = nullptr, *dw = nullptr;
    uint32_t *dtoff = nullptr, *djord = nullptr;
    hipStream_t stream = nullptr;
    // grid set by mdp_scenario_set_grid (device resident)
    int ts = 0, tdis = 0;
    uint32_t ne = 0, nc = 0, nK = 0, nd = 0;
    double *de = nullptr, *dc = nullptr, *dK = nullptr, *dsr = nullptr, *dV = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
};

namespace {

void scn_free_grid(mdp_scenario *sc)
{
    for (double **p : {&sc->de, &sc->dc, &sc->dK, &sc->dsr, &sc->dV}) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
    sc->ne = sc->nc = sc->nK = sc->nd = 0;
}

size_t scn_lds(const mdp_scenario *sc) { return (sc->nterm + 2 * (size_t)sc->ns * kE) * sizeof(double); }

// k_scn_v (which = 1), k_scn_lik (which = 2) or both (3) on stream st
int scn_launch(mdp_scenario *sc, double *dout, hipStream_t st, int which)
{
    const uint32_t nchunk = (sc->ne + kE - 1) / kE;
    ScnArgs a{sc->n, sc->ns, sc->nterm, sc->ts, sc->tdis, sc->kind, sc->ne, sc->nc, sc->nK, sc->nd,
              (uint32_t)sc->jord.size()};
    const size_t lds = scn_lds(sc);
    const size_t npt = (size_t)sc->nc * sc->nK * sc->nd;
    if (which & 1) {
        hipLaunchKernelGGL(k_scn_v, dim3(nchunk * sc->nc), dim3(kScnBlock), lds, st, a, sc->dS, sc->dtoff,
                           sc->djord, sc->dw, sc->de, sc->dc, sc->dV);
        SCN_TRY(hipGetLastError());
    }
    if (which & 2) {
        hipLaunchKernelGGL(k_scn_lik, dim3((uint32_t)(nchunk * npt)), dim3(kScnBlock), lds, st, a, sc->dS,
                           sc->dtoff, sc->djord, sc->dV, sc->de, sc->dc, sc->dK, sc->dsr, dout);
        SCN_TRY(hipGetLastError());
    }
    return MDP_OK;
}

}  // namespace

extern "C" {

double mdp_kgrid(uint32_t s, double lo, double hi, double *K)
{
    // dieoff.c:284-286 / loss.c:315-317
    for (uint32_t i = 0; i < s; ++i)
        K[i] = pow(10.0, ((double)i) / (s - 1) * (log10(hi) - log10(lo)) + log10(lo));
    return s ? K[0] : 0.0;
}

double mdp_dgrid(uint32_t s, double lo, double hi, double *dv)
{
    // loss.c:319-322
    for (uint32_t i = 0; i < s; ++i) dv[i] = i * (hi - lo) / (s - 1) + lo;
    return s ? dv[0] : 0.0;
}

int mdp_scenario_create(const int32_t *row, uint32_t n, double m, float p, double d, int kind, int device,
                        mdp_scenario **out)
{
    if (!row || !out || n == 0) return mdp_set_error(MDP_EINVAL, "null argument");
    *out = nullptr;
    if (n > kMaxN)
        return mdp_set_error(MDP_EUNSUPPORTED, "%u patches: the scenario engine holds 3^n Pc entries in LDS (n <= %u)",
                             n, kMaxN);
    for (uint32_t j = 0; j < n; ++j)
        if (row[j] < -1 || row[j] > 1) return mdp_set_error(MDP_EINVAL, "observation %d not in {-1,0,1}", row[j]);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return mdp_set_error(MDP_ENODEV, "no HIP device available");
    if (device < 0 || device >= ndev) return mdp_set_error(MDP_ENODEV, "device %d not present", device);
    mdp_scenario *sc = new (std::nothrow) mdp_scenario();
    if (!sc) return mdp_set_error(MDP_ENOMEM, "out of host memory");
    sc->n = n;
    sc->ns = 1u << n;
    sc->kind = kind;
    sc->m = m;
    sc->d = d;
    sc->device = device;
    const uint32_t ns = sc->ns;
    // dispersal M (dieoff.c:238-248) and colonisation sums S[j][k] =
    // sum over l != k, ascending, of M[l][k] * j_l (dieoff.c:72-77)
    std::vector<double> M((size_t)n * n, 0.0);
    const double a = 1.0 / m;
    for (uint32_t i = 0; i < n; ++i)
        for (uint32_t j = i + 1; j < n; ++j) M[i * n + j] = M[j * n + i] = exp(-a * (double)(j - i) * d);
    sc->S.assign((size_t)ns * n, 0.0);
    for (uint32_t j = 0; j < ns; ++j)
        for (uint32_t k = 0; k < n; ++k) {
            double s1 = 0;
            for (uint32_t l = 0; l < n; ++l)
                if (l != k) s1 += M[l * n + k] * (double)((j >> (n - 1 - l)) & 1u);
            sc->S[(size_t)j * n + k] = s1;
        }
    // observed first-row states and float priors (dieoff.c:198-232):
    // w[s] = prior of s
    sc->w.assign(ns, 0.0);
    {
        uint32_t nm = 0;
        for (uint32_t j = 0; j < n; ++j) nm += row[j] == -1;
        const uint32_t np = 1u << nm;
        std::vector<uint32_t> ps(np, 0);
        std::vector<float> pr(np, 1.0f);
        uint32_t s1 = 0;
        for (uint32_t j = 0; j < n; ++j) {
            if (row[j] == -1) s1++;
            for (uint32_t k = 0; k < np; ++k) {
                if (row[j] > -1) {
                    ps[k] += (uint32_t)row[j] << (n - j - 1);
                } else {
                    const uint32_t st1 = np >> s1, bitv = k / st1 % 2;
                    ps[k] += bitv << (n - j - 1);
                    pr[k] *= (float)bitv * p + (float)(1 - bitv) * (1 - p);
                }
            }
        }
        for (uint32_t k = 0; k < np; ++k) sc->w[ps[k]] += (double)pr[k];
    }
    // Pc table layout: rows j (ascending), supersets ascending; j rows in
    // popcount order for the lane-uniform product
    sc->toff.resize(ns);
    uint32_t off = 0;
    for (uint32_t j = 0; j < ns; ++j) {
        sc->toff[j] = off;
        off += 1u << (n - __builtin_popcount(j));
    }
    sc->nterm = off;
    // row schedule: rows dealt to the kJPar lane groups by longest-processing-
    // time-first (row j costs 2^(n - |j|) terms; 99.5 % balanced for n = 8),
    // stored so that group g runs jord[g], jord[g + kJPar], ...; short
    // groups are padded with ns (skipped)
    {
        std::vector<uint32_t> rows(ns);
        for (uint32_t j = 0; j < ns; ++j) rows[j] = j;
        std::stable_sort(rows.begin(), rows.end(),
                         [](uint32_t x, uint32_t y) { return __builtin_popcount(x) < __builtin_popcount(y); });
        std::vector<std::vector<uint32_t>> grp(kJPar);
        std::vector<uint64_t> load(kJPar, 0);
        for (uint32_t j : rows) {
            const uint32_t g = (uint32_t)(std::min_element(load.begin(), load.end()) - load.begin());
            grp[g].push_back(j);
            load[g] += 1ull << (n - __builtin_popcount(j));
        }
        size_t mx = 0;
        for (auto &v : grp) mx = std::max(mx, v.size());
        sc->jord.assign(mx * kJPar, ns);
        for (uint32_t g = 0; g < (uint32_t)kJPar; ++g)
            for (size_t i = 0; i < grp[g].size(); ++i) sc->jord[i * kJPar + g] = grp[g][i];
    }
    int rc;
    if (hipSetDevice(device) != hipSuccess) {
        delete sc;
        return mdp_set_error(MDP_EHIP, "hipSetDevice(%d) failed", device);
    }
    if ((rc = dev_up(&sc->dS, sc->S)) || (rc = dev_up(&sc->dw, sc->w)) || (rc = dev_up(&sc->dtoff, sc->toff)) ||
        (rc = dev_up(&sc->djord, sc->jord)) || hipStreamCreateWithFlags(&sc->stream, hipStreamNonBlocking) != hipSuccess) {
        mdp_scenario_destroy(sc);
        return rc ? rc : mdp_set_error(MDP_EHIP, "stream creation failed");
    }
    const size_t lds = (sc->nterm + 2 * (size_t)ns * kE) * sizeof(double);
    if (lds > 64 * 1024) {
        (void)hipFuncSetAttribute((const void *)k_scn_v, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        (void)hipFuncSetAttribute((const void *)k_scn_lik, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    }
    *out = sc;
    return MDP_OK;
}

void mdp_scenario_destroy(mdp_scenario *sc)
{
    if (!sc) return;
    (void)hipSetDevice(sc->device);
    if (sc->stream) (void)hipStreamSynchronize(sc->stream);
    scn_free_grid(sc);
    for (void *p : {(void *)sc->dS, (void *)sc->dw, (void *)sc->dtoff, (void *)sc->djord})
        if (p) (void)hipFree(p);
    if (sc->ev0) (void)hipEventDestroy(sc->ev0);
    if (sc->ev1) (void)hipEventDestroy(sc->ev1);
    if (sc->stream) (void)hipStreamDestroy(sc->stream);
    delete sc;
}

int mdp_scenario_set_grid(mdp_scenario *sc, int ts, int tdis, const double *e, uint32_t ne, const double *c,
                          uint32_t nc, const double *K, uint32_t nK, const double *dsrc, uint32_t nd)
{
    if (!sc || (ne && !e) || (nc && !c) || (nK && !K)) return mdp_set_error(MDP_EINVAL, "null argument");
    if (ts < 0 || tdis < 0) return mdp_set_error(MDP_EINVAL, "negative number of years");
    if (sc->kind == 1) {
        if (nd && !dsrc) return mdp_set_error(MDP_EINVAL, "null source distances");
    } else {
        nd = 1;
    }
    SCN_TRY(hipSetDevice(sc->device));
    SCN_TRY(hipStreamSynchronize(sc->stream));
    scn_free_grid(sc);
    sc->ts = ts, sc->tdis = tdis;
    if (!ne || !nc || !nK || !nd) return MDP_OK;
    const uint32_t n = sc->n, ns = sc->ns;
    const uint32_t nchunk = (ne + kE - 1) / kE;
    if ((size_t)nchunk * nc * nK * nd > 0x7fffffffull)
        return mdp_set_error(MDP_EUNSUPPORTED, "grid of %zu points too large", (size_t)ne * nc * nK * nd);
    // source terms M[n][k] = exp(-a (k+1) dsrc), loss.c:365
    std::vector<double> src((size_t)nd * n, 0.0);
    if (sc->kind == 1)
        for (uint32_t id = 0; id < nd; ++id)
            for (uint32_t k = 0; k < n; ++k) src[(size_t)id * n + k] = exp(-(1.0 / sc->m) * (k + 1) * dsrc[id]);
    if (hipMalloc((void **)&sc->de, ne * sizeof(double)) != hipSuccess ||
        hipMalloc((void **)&sc->dc, nc * sizeof(double)) != hipSuccess ||
        hipMalloc((void **)&sc->dK, nK * sizeof(double)) != hipSuccess ||
        hipMalloc((void **)&sc->dsr, std::max<size_t>(1, src.size()) * sizeof(double)) != hipSuccess ||
        hipMalloc((void **)&sc->dV, (size_t)nc * nchunk * ns * kE * sizeof(double)) != hipSuccess) {
        scn_free_grid(sc);
        return mdp_set_error(MDP_ENOMEM, "device allocation failed");
    }
    if (hipMemcpy(sc->de, e, ne * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(sc->dc, c, nc * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(sc->dK, K, nK * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
        (!src.empty() &&
         hipMemcpy(sc->dsr, src.data(), src.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)) {
        scn_free_grid(sc);
        return mdp_set_error(MDP_EHIP, "upload failed");
    }
    sc->ne = ne, sc->nc = nc, sc->nK = nK, sc->nd = nd;
    return MDP_OK;
}

int mdp_scenario_run(mdp_scenario *sc, double *d_out, void *stream)
{
    if (!sc) return mdp_set_error(MDP_EINVAL, "null scenario");
    if (!sc->ne) return MDP_OK;
    if (!d_out) return mdp_set_error(MDP_EINVAL, "null device output");
    SCN_TRY(hipSetDevice(sc->device));
    return scn_launch(sc, d_out, stream ? (hipStream_t)stream : sc->stream, 3);
}

int mdp_scenario_time_kernels(mdp_scenario *sc, double *d_out, void *stream, int reps, double *ms)
{
    if (!sc || !ms || reps <= 0) return mdp_set_error(MDP_EINVAL, "bad timing request");
    if (!sc->ne) return mdp_set_error(MDP_EINVAL, "no grid set");
    SCN_TRY(hipSetDevice(sc->device));
    hipStream_t st = stream ? (hipStream_t)stream : sc->stream;
    if (!sc->ev0) SCN_TRY(hipEventCreate(&sc->ev0));
    if (!sc->ev1) SCN_TRY(hipEventCreate(&sc->ev1));
    int rc = scn_launch(sc, d_out, st, 3);
    if (rc) return rc;
    for (int which = 1; which <= 2; ++which) {
        SCN_TRY(hipEventRecord(sc->ev0, st));
        for (int i = 0; i < reps; ++i)
            if ((rc = scn_launch(sc, d_out, st, which))) return rc;
        SCN_TRY(hipEventRecord(sc->ev1, st));
        SCN_TRY(hipEventSynchronize(sc->ev1));
        float t = 0;
        SCN_TRY(hipEventElapsedTime(&t, sc->ev0, sc->ev1));
        ms[which - 1] = (double)t / reps;
    }
    return MDP_OK;
}

int mdp_scenario_lik(mdp_scenario *sc, int ts, int tdis, const double *e, uint32_t ne, const double *c,
                     uint32_t nc, const double *K, uint32_t nK, const double *dsrc, uint32_t nd, double *out)
{
    if (!sc || !out) return mdp_set_error(MDP_EINVAL, "null argument");
    int rc = mdp_scenario_set_grid(sc, ts, tdis, e, ne, c, nc, K, nK, dsrc, nd);
    if (rc || !sc->ne) return rc;
    const size_t npts = (size_t)sc->ne * sc->nc * sc->nK * sc->nd;
    double *dout = nullptr;
    if (hipMalloc((void **)&dout, npts * sizeof(double)) != hipSuccess)
        return mdp_set_error(MDP_ENOMEM, "device allocation failed");
    rc = scn_launch(sc, dout, sc->stream, 3);
    if (!rc && (hipMemcpyAsync(out, dout, npts * sizeof(double), hipMemcpyDeviceToHost, sc->stream) != hipSuccess ||
                hipStreamSynchronize(sc->stream) != hipSuccess))
        rc = mdp_set_error(MDP_EHIP, "scenario run failed");
    (void)hipFree(dout);
    return rc;
}

}  // extern "C"
