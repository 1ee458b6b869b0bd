// midaspom_amd/csrc/spom_engine.hip -- MI355X (gfx950) posterior-grid
// likelihood engine for the stochastic patch occupancy model.
//
// Replaces the reference hot loop /root/reference/sources/main_MIDASPOM.c:341-395
// (colonisation pressure :350-358, compPePc :18-50, P = Pe*Pc dgemm :363,
// forward propagation :368-384, prior sum + log :386-392).
//
// Factorisation used.  For observed short states a -> b with
// bit sets A, B and hidden intermediate state j (extinction first, then
// colonisation), the reference forms P[a][b] = sum_j Pe[a][j] Pc[j][b] with
//   Pe[a][j] = [j <= A] x^{|A|-|j|} y^{|j|}        (x = min(e,1), y = 1-x)
//   Pc[j][b] = [j <= B] prod_{k : j_k = 0} (B_k ? pC_jk : 1-pC_jk),
//   pC_jk    = min(1, c * S[j][k]),  S = grid-invariant dispersal sums.
// Pe depends on e only through |j| and Pc on c only, so
//   P[a][b](e,c) = sum_{m=0}^{|A&B|} x^{|A|-m} y^m Q_ab[m](c),
//   Q_ab[m](c)   = sum_{j <= A&B, |j| = m} Pc[j][b](c).
// Kernels:
//   k_colsum     (once per engine) S[k][j]
//   k_coltables  (per c)  Z[c][j] = prod_{non-var k}(1-pC_jk), PV[c][b][j] = pC_j,var(b)
//   k_coefs      (per c)  Q[c][pair][m]
//   k_forward    (per (e,c) point) forward recursion over the years with the
//                transition entries evaluated from Q in Bernstein/Horner form;
//                lanes = e values, one c per workgroup so Q is wave-uniform
//                and streams through the scalar cache (s_load), no LDS.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <new>
#include <vector>

#include "mdp_internal.h"

namespace {

constexpr int kBlock = 256;
constexpr uint32_t kOffBits = 22;              // coefficient offset bits in a use descriptor
constexpr uint32_t kOffMask = (1u << kOffBits) - 1u;
constexpr int kColTile = 8;                    // c values per k_coltables thread

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return mdp_set_error(MDP_EHIP, "%s failed: %s (%s:%d)", #expr,               \
                                 hipGetErrorString(e_), __FILE__, __LINE__);              \
    } while (0)

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------

// S[k][j] = sum over set bits of state j (ascending variable column l, l != k)
// of M[l][k] -- the reference's per-point sum at :350-357, which skips zero
// terms exactly, so the result is bit-identical.
__global__ __launch_bounds__(kBlock) void k_colsum(const double *__restrict__ M,
                                                   const uint32_t *__restrict__ var_cols,
                                                   uint32_t n, uint32_t nvar, uint32_t nstates,
                                                   double *__restrict__ S)
{
    const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t k = blockIdx.y;
    if (j >= nstates) return;
    double acc = 0.0;
    for (uint32_t b = 0; b < nvar; ++b) {
        const uint32_t col = var_cols[b];
        if (((j >> (nvar - 1 - b)) & 1u) && col != k) acc += M[(size_t)col * n + k];
    }
    S[(size_t)k * nstates + j] = acc;
}

// Per c value: Z[c][j] (product over always-zero columns, ascending) and the
// clamped pressure on each variable column.  One thread = one hidden state j
// for kColTile consecutive c values (S is read once per tile).
__global__ __launch_bounds__(kBlock) void k_coltables(
    const double *__restrict__ S, uint32_t nstates, const uint32_t *__restrict__ nonvar,
    uint32_t nnv, const uint32_t *__restrict__ var_cols, uint32_t nvar,
    const double *__restrict__ cvals, uint32_t nc, double *__restrict__ Z, double *__restrict__ PV)
{
    const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t c0 = blockIdx.y * kColTile;
    if (j >= nstates) return;
    double c[kColTile], z[kColTile];
#pragma unroll
    for (int t = 0; t < kColTile; ++t) {
        c[t] = (c0 + t < nc) ? cvals[c0 + t] : 0.0;
        z[t] = 1.0;
    }
    for (uint32_t q = 0; q < nnv; ++q) {
        const double s = S[(size_t)nonvar[q] * nstates + j];
#pragma unroll
        for (int t = 0; t < kColTile; ++t) {
            double pc = c[t] * s;
            pc = pc > 1.0 ? 1.0 : pc;
            z[t] = z[t] * (1.0 - pc);
        }
    }
#pragma unroll
    for (int t = 0; t < kColTile; ++t)
        if (c0 + t < nc) Z[(size_t)(c0 + t) * nstates + j] = z[t];
    for (uint32_t b = 0; b < nvar; ++b) {
        const double s = S[(size_t)var_cols[b] * nstates + j];
#pragma unroll
        for (int t = 0; t < kColTile; ++t) {
            if (c0 + t < nc) {
                double pc = c[t] * s;
                pc = pc > 1.0 ? 1.0 : pc;
                PV[((size_t)(c0 + t) * nvar + b) * nstates + j] = pc;
            }
        }
    }
}

// Q[c][off_p + m] = sum_{j <= A&B, |j| = m} Z[c][j] * prod_{var b, j_b = 0} f_b,
// f_b = B_b ? pC : 1 - pC (ascending variable column, as compPePc's k loop).
__global__ __launch_bounds__(kBlock) void k_coefs(
    const uint32_t *__restrict__ pairA, const uint32_t *__restrict__ pairB,
    const uint32_t *__restrict__ pairOff, uint32_t npairs, uint32_t nvar, uint32_t nstates,
    const double *__restrict__ Z, const double *__restrict__ PV, uint32_t ncoef,
    double *__restrict__ Q)
{
    const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t ic = blockIdx.y;
    if (p >= npairs) return;
    const uint32_t A = pairA[p], B = pairB[p], X = A & B;
    const uint32_t nX = __popc(X);
    const double *z = Z + (size_t)ic * nstates;
    const double *pv = PV + (size_t)ic * nvar * nstates;
    double *q = Q + (size_t)ic * ncoef + pairOff[p];
    for (uint32_t m = 0; m <= nX; ++m) {
        double acc = 0.0;
        uint32_t sub = X;
        for (;;) {
            if ((uint32_t)__popc(sub) == m) {
                double prod = z[sub];
                for (uint32_t b = 0; b < nvar; ++b) {
                    const uint32_t bit = nvar - 1 - b;
                    if (!((sub >> bit) & 1u)) {
                        const double f = pv[(size_t)b * nstates + sub];
                        prod *= ((B >> bit) & 1u) ? f : 1.0 - f;
                    }
                }
                acc += prod;
            }
            if (sub == 0) break;
            sub = (sub - 1) & X;
        }
        q[m] = acc;
    }
}

// Transition entry P[a][b](e,c) from its coefficient block (wave-uniform
// pointer -> scalar loads): Horner in x with y^m folded in, then x^{|A|-|X|}.
__device__ __forceinline__ double eval_transition(const double *__restrict__ q, uint32_t d,
                                                  double x, double y)
{
    const double *cf = q + (d & kOffMask);
    const uint32_t nX = (d >> kOffBits) & 31u;
    const uint32_t nA = d >> 27;
    double acc = cf[0];
    double yp = 1.0;
    for (uint32_t m = 1; m <= nX; ++m) {
        yp *= y;
        acc = fma(acc, x, cf[m] * yp);
    }
    for (uint32_t r = nX; r < nA; ++r) acc *= x;
    return acc;
}

// Forward recursion for one grid point per lane.  Q3 semantics of the
// reference (:368-369): start from a vector of ones over the year-0 states,
// L = prior0 * sum_l v[l] accumulated as sum_l v[l]*prior0.
template <int NPMAX>
__global__ __launch_bounds__(kBlock) void k_forward(
    const double *__restrict__ Q, uint32_t ncoef, const uint32_t *__restrict__ desc,
    const uint32_t *__restrict__ npy, uint32_t tmax, double prior0,
    const double *__restrict__ evals, uint32_t ne, double *__restrict__ out, uint32_t ld_out)
{
    const uint32_t ic = blockIdx.x;
    const uint32_t ie = blockIdx.y * kBlock + threadIdx.x;
    const bool active = ie < ne;
    const double e = active ? evals[ie] : 0.0;
    const double x = e > 1.0 ? 1.0 : e;
    const double y = 1.0 - x;
    const double *__restrict__ q = Q + (size_t)ic * ncoef;

    double v[NPMAX];
    uint32_t npp = npy[0];
#pragma unroll
    for (int k = 0; k < NPMAX; ++k) v[k] = (uint32_t)k < npp ? 1.0 : 0.0;
    uint32_t u = 0;
    for (uint32_t t = 1; t < tmax; ++t) {
        const uint32_t npc = npy[t];
        double vn[NPMAX];
#pragma unroll
        for (int l = 0; l < NPMAX; ++l) {
            double acc = 0.0;
            if ((uint32_t)l < npc) {
#pragma unroll
                for (int k = 0; k < NPMAX; ++k) {
                    if ((uint32_t)k < npp) {
                        const double P = eval_transition(q, desc[u], x, y);
                        ++u;
                        acc = fma(v[k], P, acc);
                    }
                }
            }
            vn[l] = acc;
        }
#pragma unroll
        for (int l = 0; l < NPMAX; ++l) v[l] = vn[l];
        npp = npc;
    }
    double L = 0.0;
#pragma unroll
    for (int l = 0; l < NPMAX; ++l)
        if ((uint32_t)l < npp) L += v[l] * prior0;
    if (active) out[(size_t)ie * ld_out + ic] = log(L);
}

// ---------------------------------------------------------------------------
// engine
// ---------------------------------------------------------------------------

template <typename T>
int dev_alloc(T **p, size_t count)
{
    *p = nullptr;
    if (count == 0) count = 1;
    hipError_t e = hipMalloc((void **)p, count * sizeof(T));
    if (e != hipSuccess)
        return mdp_set_error(MDP_ENOMEM, "hipMalloc(%zu bytes) failed: %s", count * sizeof(T),
                             hipGetErrorString(e));
    return MDP_OK;
}

template <typename T>
int dev_upload(T **p, const std::vector<T> &h)
{
    int rc = dev_alloc(p, h.size());
    if (rc) return rc;
    if (!h.empty()) HIP_TRY(hipMemcpy(*p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return MDP_OK;
}

template <typename T>
int dev_reserve(T **p, size_t *cap, size_t count)
{
    if (count <= *cap && *p) return MDP_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    int rc = dev_alloc(p, count);
    if (rc) return rc;
    *cap = count;
    return MDP_OK;
}

enum { kEvBegin = 0, kEvColTables, kEvCoefs, kEvForward, kNumEv };
const char *const kKernelNames[] = {"k_coltables", "k_coefs", "k_forward"};

struct DevCtx {
    int device = 0;
    hipStream_t stream = nullptr;
    double *S = nullptr;
    uint32_t *var_cols = nullptr, *nonvar = nullptr;
    uint32_t *pairA = nullptr, *pairB = nullptr, *pairOff = nullptr;
    uint32_t *desc = nullptr, *npy = nullptr;
    double *e = nullptr, *c = nullptr;
    size_t cap_e = 0, cap_c = 0;
    uint32_t ne = 0, nc = 0;
    double *Z = nullptr, *PV = nullptr, *Q = nullptr, *out = nullptr;
    size_t cap_z = 0, cap_pv = 0, cap_q = 0, cap_out = 0;
    std::vector<hipEvent_t> ev;   // kNumEv events per profiled run, reused
    size_t ev_used = 0;           // event sets recorded since the last collect
};

}  // namespace

struct mdp_engine {
    uint32_t n = 0, tmax = 0, nvar = 0, nstates = 0, nextid = 0;
    uint32_t npairs = 0, nuses = 0, ncoef = 0, npmax = 1, variant = 0;
    double prior0 = 1.0;
    std::vector<uint32_t> np, pairA, pairB, pairOff, desc;
    std::vector<DevCtx> devs;
    int profiling = 0;
    double last_ms[3] = {0, 0, 0};  // mean per run over the last collected runs
    int nlast = 0;
    uint64_t runs_collected = 0;
};

namespace {

int select_variant(uint32_t npmax, uint32_t *variant)
{
    if (npmax <= 1) *variant = 1;
    else if (npmax <= 2) *variant = 2;
    else if (npmax <= 4) *variant = 4;
    else if (npmax <= 8) *variant = 8;
    else if (npmax <= 16) *variant = 16;
    else
        return mdp_set_error(MDP_EUNSUPPORTED,
                             "a year with %u possible states (more than 4 missing patches) "
                             "exceeds the register-resident forward kernel (max 16)", npmax);
    return MDP_OK;
}

// host plan: distinct transition pairs, coefficient offsets, use descriptors
int build_plan(mdp_engine *eng, const mdp_problem *p)
{
    eng->n = p->n;
    eng->tmax = p->tmax;
    eng->nvar = p->nvar;
    eng->nextid = p->nextid;
    if (p->nvar > 24)
        return mdp_set_error(MDP_EUNSUPPORTED, "%u variable columns (engine limit 24)", p->nvar);
    eng->nstates = 1u << p->nvar;
    eng->prior0 = (double)p->prior[0];
    eng->np.resize(p->tmax);
    eng->npmax = 1;
    for (uint32_t t = 0; t < p->tmax; ++t) {
        eng->np[t] = p->year_off[t + 1] - p->year_off[t];
        eng->npmax = std::max(eng->npmax, eng->np[t]);
    }
    int rc = select_variant(eng->npmax, &eng->variant);
    if (rc) return rc;
    std::map<uint64_t, uint32_t> pair_index;
    uint32_t off = 0;
    for (uint32_t t = 1; t < p->tmax; ++t) {
        const uint32_t *prev = p->year_ids + p->year_off[t - 1];
        const uint32_t *cur = p->year_ids + p->year_off[t];
        for (uint32_t l = 0; l < eng->np[t]; ++l)
            for (uint32_t k = 0; k < eng->np[t - 1]; ++k) {
                const uint32_t a = prev[k], b = cur[l];
                if (a >= p->nextid || b >= p->nextid)
                    return mdp_set_error(MDP_EINVAL, "short id out of range in year %u", t);
                const uint64_t key = ((uint64_t)a << 32) | b;
                auto it = pair_index.find(key);
                uint32_t pi;
                if (it == pair_index.end()) {
                    pi = (uint32_t)eng->pairA.size();
                    pair_index.emplace(key, pi);
                    const uint32_t A = p->short_state[a], B = p->short_state[b];
                    eng->pairA.push_back(A);
                    eng->pairB.push_back(B);
                    eng->pairOff.push_back(off);
                    off += (uint32_t)__builtin_popcount(A & B) + 1u;
                    if (off > kOffMask)
                        return mdp_set_error(MDP_EUNSUPPORTED, "too many transition coefficients");
                } else {
                    pi = it->second;
                }
                const uint32_t A = eng->pairA[pi], B = eng->pairB[pi];
                const uint32_t nA = (uint32_t)__builtin_popcount(A);
                const uint32_t nX = (uint32_t)__builtin_popcount(A & B);
                eng->desc.push_back(eng->pairOff[pi] | (nX << kOffBits) | (nA << 27));
            }
    }
    eng->npairs = (uint32_t)eng->pairA.size();
    eng->nuses = (uint32_t)eng->desc.size();
    eng->ncoef = off;
    return MDP_OK;
}

int init_device(mdp_engine *eng, DevCtx &d, const mdp_problem *p)
{
    HIP_TRY(hipSetDevice(d.device));
    HIP_TRY(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
    std::vector<uint32_t> var(p->var_cols, p->var_cols + p->nvar), nonvar;
    std::vector<uint8_t> isvar(p->n, 0);
    for (uint32_t b = 0; b < p->nvar; ++b) isvar[p->var_cols[b]] = 1;
    for (uint32_t k = 0; k < p->n; ++k)
        if (!isvar[k]) nonvar.push_back(k);
    std::vector<double> M(p->M, p->M + (size_t)p->n * p->n);
    double *dM = nullptr;
    int rc;
    if ((rc = dev_upload(&dM, M))) return rc;
    if ((rc = dev_upload(&d.var_cols, var)) || (rc = dev_upload(&d.nonvar, nonvar)) ||
        (rc = dev_upload(&d.pairA, eng->pairA)) || (rc = dev_upload(&d.pairB, eng->pairB)) ||
        (rc = dev_upload(&d.pairOff, eng->pairOff)) || (rc = dev_upload(&d.desc, eng->desc)) ||
        (rc = dev_upload(&d.npy, eng->np)) ||
        (rc = dev_alloc(&d.S, (size_t)p->n * eng->nstates))) {
        (void)hipFree(dM);
        return rc;
    }
    dim3 grid((eng->nstates + kBlock - 1) / kBlock, p->n);
    hipLaunchKernelGGL(k_colsum, grid, dim3(kBlock), 0, d.stream, dM, d.var_cols, p->n, p->nvar,
                       eng->nstates, d.S);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(d.stream));
    (void)hipFree(dM);
    return MDP_OK;
}

void free_device(DevCtx &d)
{
    (void)hipSetDevice(d.device);
    void *ptrs[] = {d.S, d.var_cols, d.nonvar, d.pairA, d.pairB, d.pairOff, d.desc, d.npy,
                    d.e, d.c, d.Z, d.PV, d.Q, d.out};
    for (void *ptr : ptrs)
        if (ptr) (void)hipFree(ptr);
    for (hipEvent_t ev : d.ev) (void)hipEventDestroy(ev);
    if (d.stream) (void)hipStreamDestroy(d.stream);
}

int set_grid_dev(mdp_engine *eng, DevCtx &d, const double *e, uint32_t ne, const double *c,
                 uint32_t nc)
{
    HIP_TRY(hipSetDevice(d.device));
    int rc;
    if ((rc = dev_reserve(&d.e, &d.cap_e, ne)) || (rc = dev_reserve(&d.c, &d.cap_c, nc)) ||
        (rc = dev_reserve(&d.Z, &d.cap_z, (size_t)nc * eng->nstates)) ||
        (rc = dev_reserve(&d.PV, &d.cap_pv, (size_t)nc * eng->nvar * eng->nstates)) ||
        (rc = dev_reserve(&d.Q, &d.cap_q, (size_t)nc * eng->ncoef)))
        return rc;
    if (ne) HIP_TRY(hipMemcpy(d.e, e, ne * sizeof(double), hipMemcpyHostToDevice));
    if (nc) HIP_TRY(hipMemcpy(d.c, c, nc * sizeof(double), hipMemcpyHostToDevice));
    d.ne = ne;
    d.nc = nc;
    return MDP_OK;
}

int launch_forward(mdp_engine *eng, DevCtx &d, double *out, uint32_t ld, hipStream_t s)
{
    dim3 grid(d.nc, (d.ne + kBlock - 1) / kBlock);
    switch (eng->variant) {
#define MDP_FWD(NP)                                                                          \
    case NP:                                                                                 \
        hipLaunchKernelGGL(k_forward<NP>, grid, dim3(kBlock), 0, s, d.Q, eng->ncoef, d.desc, \
                           d.npy, eng->tmax, eng->prior0, d.e, d.ne, out, ld);               \
        break;
        MDP_FWD(1) MDP_FWD(2) MDP_FWD(4) MDP_FWD(8) MDP_FWD(16)
#undef MDP_FWD
    default:
        return mdp_set_error(MDP_EUNSUPPORTED, "no forward kernel variant %u", eng->variant);
    }
    HIP_TRY(hipGetLastError());
    return MDP_OK;
}

int run_dev(mdp_engine *eng, DevCtx &d, double *out, uint32_t ld, hipStream_t s)
{
    HIP_TRY(hipSetDevice(d.device));
    if (d.ne == 0 || d.nc == 0) return MDP_OK;
    if (d.ne > 65535u * kBlock || d.nc > 0x7fffffffu)
        return mdp_set_error(MDP_EUNSUPPORTED, "grid %u x %u too large", d.ne, d.nc);
    const bool prof = eng->profiling != 0;
    hipEvent_t *ev = nullptr;
    if (prof) {
        if ((d.ev_used + 1) * kNumEv > d.ev.size()) {
            for (int i = 0; i < kNumEv; ++i) {
                hipEvent_t x;
                HIP_TRY(hipEventCreate(&x));
                d.ev.push_back(x);
            }
        }
        ev = &d.ev[d.ev_used * kNumEv];
        ++d.ev_used;
        HIP_TRY(hipEventRecord(ev[kEvBegin], s));
    }
    {
        dim3 grid((eng->nstates + kBlock - 1) / kBlock, (d.nc + kColTile - 1) / kColTile);
        hipLaunchKernelGGL(k_coltables, grid, dim3(kBlock), 0, s, d.S, eng->nstates, d.nonvar,
                           eng->n - eng->nvar, d.var_cols, eng->nvar, d.c, d.nc, d.Z, d.PV);
        HIP_TRY(hipGetLastError());
    }
    if (prof) HIP_TRY(hipEventRecord(ev[kEvColTables], s));
    if (eng->npairs) {
        dim3 grid((eng->npairs + kBlock - 1) / kBlock, d.nc);
        hipLaunchKernelGGL(k_coefs, grid, dim3(kBlock), 0, s, d.pairA, d.pairB, d.pairOff,
                           eng->npairs, eng->nvar, eng->nstates, d.Z, d.PV, eng->ncoef, d.Q);
        HIP_TRY(hipGetLastError());
    }
    if (prof) HIP_TRY(hipEventRecord(ev[kEvCoefs], s));
    int rc = launch_forward(eng, d, out, ld, s);
    if (rc) return rc;
    if (prof) HIP_TRY(hipEventRecord(ev[kEvForward], s));
    return MDP_OK;
}

// Mean kernel durations over every profiled run since the last collect.
int collect_times(mdp_engine *eng, DevCtx &d)
{
    if (d.ev_used == 0) return MDP_OK;
    HIP_TRY(hipSetDevice(d.device));
    HIP_TRY(hipEventSynchronize(d.ev[(d.ev_used - 1) * kNumEv + kEvForward]));
    double sum[3] = {0, 0, 0};
    for (size_t r = 0; r < d.ev_used; ++r)
        for (int k = 0; k < 3; ++k) {
            float ms = 0;
            HIP_TRY(hipEventElapsedTime(&ms, d.ev[r * kNumEv + k], d.ev[r * kNumEv + k + 1]));
            sum[k] += ms;
        }
    for (int k = 0; k < 3; ++k) eng->last_ms[k] = sum[k] / (double)d.ev_used;
    eng->nlast = 3;
    eng->runs_collected = d.ev_used;
    d.ev_used = 0;
    return MDP_OK;
}

}  // namespace

extern "C" {

int mdp_engine_create(const mdp_problem *p, const int *devices, int n_devices, mdp_engine **out)
{
    if (!p || !out || n_devices < 0) return mdp_set_error(MDP_EINVAL, "null argument");
    *out = nullptr;
    if (p->n == 0 || p->tmax == 0 || !p->M || !p->year_off || !p->year_ids || !p->prior ||
        !p->short_state || (p->nvar && !p->var_cols))
        return mdp_set_error(MDP_EINVAL, "incomplete problem description");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return mdp_set_error(MDP_ENODEV, "no HIP device available");
    mdp_engine *eng = new (std::nothrow) mdp_engine();
    if (!eng) return mdp_set_error(MDP_ENOMEM, "out of host memory");
    int rc = build_plan(eng, p);
    if (rc) {
        delete eng;
        return rc;
    }
    std::vector<int> ids;
    if (n_devices == 0) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        ids.push_back(cur);
    } else {
        for (int i = 0; i < n_devices; ++i) ids.push_back(devices ? devices[i] : i);
    }
    for (int id : ids)
        if (id < 0 || id >= ndev) {
            delete eng;
            return mdp_set_error(MDP_ENODEV, "device %d not present (%d visible)", id, ndev);
        }
    eng->devs.resize(ids.size());
    for (size_t i = 0; i < ids.size(); ++i) {
        eng->devs[i].device = ids[i];
        rc = init_device(eng, eng->devs[i], p);
        if (rc) {
            mdp_engine_destroy(eng);
            return rc;
        }
    }
    *out = eng;
    return MDP_OK;
}

void mdp_engine_destroy(mdp_engine *eng)
{
    if (!eng) return;
    for (auto &d : eng->devs) free_device(d);
    delete eng;
}

int mdp_engine_set_grid(mdp_engine *eng, const double *e, uint32_t ne, const double *c, uint32_t nc)
{
    if (!eng || (ne && !e) || (nc && !c)) return mdp_set_error(MDP_EINVAL, "null argument");
    if (eng->devs.size() != 1)
        return mdp_set_error(MDP_EINVAL, "mdp_engine_set_grid needs a single-device engine");
    return set_grid_dev(eng, eng->devs[0], e, ne, c, nc);
}

int mdp_engine_run(mdp_engine *eng, double *d_out, uint32_t ld_out, void *stream)
{
    if (!eng || !d_out) return mdp_set_error(MDP_EINVAL, "null argument");
    if (eng->devs.size() != 1)
        return mdp_set_error(MDP_EINVAL, "mdp_engine_run needs a single-device engine");
    DevCtx &d = eng->devs[0];
    if (ld_out < d.nc) return mdp_set_error(MDP_EINVAL, "ld_out %u < nc %u", ld_out, d.nc);
    hipStream_t s = stream ? (hipStream_t)stream : d.stream;
    return run_dev(eng, d, d_out, ld_out, s);
}

int mdp_loglik_grid(mdp_engine *eng, const double *e, uint32_t ne, const double *c, uint32_t nc,
                    double *out)
{
    if (!eng || !out || (ne && !e) || (nc && !c)) return mdp_set_error(MDP_EINVAL, "null argument");
    const uint32_t nd = (uint32_t)eng->devs.size();
    const uint32_t avg = ne / nd, rem = ne % nd;
    std::vector<uint32_t> r0(nd), r1(nd);
    int rc;
    for (uint32_t r = 0; r < nd; ++r) {
        r0[r] = r == 0 ? 0 : r * avg + rem;
        r1[r] = (r + 1) * avg + rem;
        DevCtx &d = eng->devs[r];
        const uint32_t rows = r1[r] - r0[r];
        if ((rc = set_grid_dev(eng, d, e + r0[r], rows, c, nc))) return rc;
        if ((rc = dev_reserve(&d.out, &d.cap_out, (size_t)rows * nc))) return rc;
        if ((rc = run_dev(eng, d, d.out, nc, d.stream))) return rc;
    }
    for (uint32_t r = 0; r < nd; ++r) {
        DevCtx &d = eng->devs[r];
        const uint32_t rows = r1[r] - r0[r];
        HIP_TRY(hipSetDevice(d.device));
        if (rows)
            HIP_TRY(hipMemcpyAsync(out + (size_t)r0[r] * nc, d.out, (size_t)rows * nc * sizeof(double),
                                   hipMemcpyDeviceToHost, d.stream));
    }
    for (uint32_t r = 0; r < nd; ++r) {
        HIP_TRY(hipSetDevice(eng->devs[r].device));
        HIP_TRY(hipStreamSynchronize(eng->devs[r].stream));
    }
    for (uint32_t r = nd; r-- > 0;)  // device 0 last: its means are reported
        if ((rc = collect_times(eng, eng->devs[r]))) return rc;
    return MDP_OK;
}

int mdp_engine_set_profiling(mdp_engine *eng, int enable)
{
    if (!eng) return mdp_set_error(MDP_EINVAL, "null engine");
    eng->profiling = enable;
    return MDP_OK;
}

int mdp_engine_kernel_ms(mdp_engine *eng, double *ms, int max_k)
{
    if (!eng || !ms) return mdp_set_error(MDP_EINVAL, "null argument");
    if (!eng->devs.empty()) {
        int rc = collect_times(eng, eng->devs[0]);
        if (rc) return rc;
    }
    const int k = std::min(max_k, eng->nlast);
    for (int i = 0; i < k; ++i) ms[i] = eng->last_ms[i];
    return k;
}

const char *mdp_engine_kernel_name(int k)
{
    return (k >= 0 && k < 3) ? kKernelNames[k] : "";
}

int mdp_engine_get_info(const mdp_engine *eng, mdp_engine_info *info)
{
    if (!eng || !info) return mdp_set_error(MDP_EINVAL, "null argument");
    info->n_devices = (int)eng->devs.size();
    info->npairs = eng->npairs;
    info->nuses = eng->nuses;
    info->ncoef = eng->ncoef;
    info->npmax = eng->npmax;
    info->variant = eng->variant;
    return MDP_OK;
}

int mdp_engine_work(const mdp_engine *eng, uint64_t ne, uint64_t nc, double *flop_impl,
                    double *flop_survey, double *bytes_min)
{
    if (!eng) return mdp_set_error(MDP_EINVAL, "null engine");
    const double pts = (double)ne * (double)nc;
    // implemented form, per point: each use costs a (nX+1)-term dot product
    // (2(nX+1) flops), the (|A|-nX) x-power multiplies, and one FMA into v;
    // plus the final prior sum.
    double per_pt = 0;
    for (uint32_t u = 0; u < eng->nuses; ++u) {
        const uint32_t dsc = eng->desc[u];
        const double nX = (double)((dsc >> kOffBits) & 31u), nA = (double)(dsc >> 27);
        per_pt += 2.0 * (nX + 1.0) + (nA - nX) + 2.0;
    }
    per_pt += 2.0 * eng->np[eng->tmax - 1];
    if (flop_impl) *flop_impl = per_pt * pts;
    // SURVEY.md §8(d) F_alg (dense-in-j formulation)
    double fwd = 0;
    for (uint32_t t = 1; t < eng->tmax; ++t) fwd += (double)eng->np[t - 1] * eng->np[t];
    const double falg = 2.0 * eng->n * eng->nstates + (double)eng->nvar * eng->nstates * eng->nextid +
                        2.0 * eng->nstates * eng->npairs + 2.0 * eng->np[0] * fwd;
    if (flop_survey) *flop_survey = falg * pts;
    // compulsory HBM bytes: per-c coefficient blocks + e values + outputs
    if (bytes_min) *bytes_min = 8.0 * ((double)nc * eng->ncoef + (double)ne + pts);
    return MDP_OK;
}

}  // extern "C"
