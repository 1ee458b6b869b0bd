// midaspom_amd/csrc/spom_engine.hip -- MI355X (gfx950) posterior-grid
// likelihood engine for the stochastic patch occupancy model.
//
// Replaces the reference hot loop /root/reference/sources/main_MIDASPOM.c:341-395
// (colonisation pressure :350-358, compPePc :18-50, P = Pe*Pc dgemm :363,
// forward propagation :368-384, prior sum + log :386-392).
//
// Factorisation.  For observed short states a -> b with bit
// sets A, B and hidden intermediate state j (extinction first, then
// colonisation) the reference forms P[a][b] = sum_j Pe[a][j] Pc[j][b] with
//   Pe[a][j] = [j <= A] x^{|A|-|j|} y^{|j|}        (x = min(e,1), y = 1-x)
//   Pc[j][b] = [j <= B] prod_{k : j_k = 0} (B_k ? pC_jk : 1-pC_jk),
//   pC_jk    = min(1, c * S[j][k]),   S = grid-invariant dispersal sums.
// Pe depends on e only through |j| and Pc on c only, so
//   P[a][b](e,c) = sum_{m=0}^{|A&B|} x^{|A|-m} y^m Q_ab[m](c),
//   Q_ab[m](c)   = sum_{j <= A&B, |j| = m} Pc[j][b](c).
// Multiplying by (x+y)^{D-|A|} = 1 makes every transition a homogeneous
// polynomial of ONE degree D (>= every |A|) with non-negative coefficients
//   P[a][b](e,c) = sum_{r=0}^{D} R_ab[r](c) W_r(e),  W_r = x^{D-r} y^r,
//   R_ab[r]      = sum_m Q_ab[m] C(D-|A|, r-m),
// so a transition costs D+1 FMAs against per-point weights held in VGPRs and
// per-c coefficients that are wave-uniform (scalar loads, no descriptors).
//
// Kernels (per run over an ne x nc grid):
//   k_zpv      [c][j]     Z = prod_{always-zero k} (1-pC_jk), PV_b = pC_j,var(b)
//   k_coefs    one WG / c Q (subset sums, LDS) -> R in forward-use order
//   k_forward  one lane / (e,c) point x EPL: forward recursion over the years,
//              c wave-uniform, R streamed through the scalar cache.
// Once per engine: k_colsum builds S.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <new>
#include <vector>

#include "mdp_internal.h"

namespace {

constexpr int kBlock = 256;
constexpr int kZpvJ = 64;       // k_zpv: hidden states per workgroup
constexpr int kZpvSlices = 4;   // k_zpv: waves splitting the zero-column product
constexpr int kZpvCT = 2;       // k_zpv: c values per thread
constexpr int kZpvUnroll = 8;   // k_zpv: S loads in flight per lane
constexpr int kEPL = 2;         // k_forward: default grid points (e values) per lane
constexpr int kMaxDeg = 24;
constexpr unsigned kWaitLgkm0 = 0xC07F;  // s_waitcnt lgkmcnt(0), other counters untouched
constexpr size_t kLdsBudget = 120 * 1024;  // dynamic LDS of k_coefs

__constant__ double c_binom[kMaxDeg + 1][kMaxDeg + 1];

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

// S2[r][j] = S[col(r)][j]: the colonisation sum of column k = col(r) for
// hidden state j, i.e. the sum over set bits of j (ascending variable column
// l, l != k) of M[l][k] -- the reference's per-point sum (:350-357) with its
// zero terms dropped, bit-identical.  Rows are ordered always-zero columns
// first, then variable columns, so k_zpv reads them without indirection.
__global__ __launch_bounds__(kBlock) void k_colsum(const double *__restrict__ M,
                                                   const uint32_t *__restrict__ var_cols,
                                                   const uint32_t *__restrict__ row_col,
                                                   uint32_t n, uint32_t nvar, uint32_t nstates,
                                                   double *__restrict__ S2)
{
    const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t r = blockIdx.y;
    if (j >= nstates) return;
    const uint32_t k = row_col[r];
    double acc = 0.0;
    for (uint32_t b = 0; b < nvar; ++b) {
        const uint32_t col = var_cols[b];
        if (((j >> (nvar - 1 - b)) & 1u) && col != k) acc += M[(size_t)col * n + k];
    }
    S2[(size_t)r * nstates + j] = acc;
}

// ZPV[c][0][j] = prod over always-zero columns (ascending) of (1 - pC_jk);
// ZPV[c][1+b][j] = pC_j,var(b) = min(1, c S).  A workgroup covers 64 hidden
// states x kZpvCT c values; its 4 waves each take a quarter of the zero
// columns (kZpvUnroll loads in flight per lane) and the partial products are
// multiplied in slice order through LDS.
__global__ __launch_bounds__(kBlock) void k_zpv(
    const double *__restrict__ S2, uint32_t nstates, uint32_t nnv, uint32_t nvar,
    const double *__restrict__ cvals, uint32_t nc, double *__restrict__ ZPV)
{
    __shared__ double part[kZpvSlices][kZpvCT][kZpvJ];
    const uint32_t lane = threadIdx.x % kZpvJ, slice = threadIdx.x / kZpvJ;
    const uint32_t j = blockIdx.x * kZpvJ + lane;
    const uint32_t c0 = blockIdx.y * kZpvCT;
    const bool ok = j < nstates;
    const uint32_t jj = ok ? j : 0;
    double c[kZpvCT], z[kZpvCT];
#pragma unroll
    for (int t = 0; t < kZpvCT; ++t) {
        c[t] = (c0 + t < nc) ? cvals[c0 + t] : 0.0;
        z[t] = 1.0;
    }
    const uint32_t per = (nnv + kZpvSlices - 1) / kZpvSlices;
    const uint32_t q0 = slice * per, q1 = min(nnv, q0 + per);
    uint32_t q = q0;
    for (; q + kZpvUnroll <= q1; q += kZpvUnroll) {
        double sv[kZpvUnroll];
#pragma unroll
        for (int u = 0; u < kZpvUnroll; ++u) sv[u] = S2[(size_t)(q + u) * nstates + jj];
#pragma unroll
        for (int u = 0; u < kZpvUnroll; ++u)
#pragma unroll
            for (int t = 0; t < kZpvCT; ++t)
                // 1 - min(1, c s), evaluated as max(0, 1 - c s) with one rounding
                z[t] *= fmax(0.0, fma(-c[t], sv[u], 1.0));
    }
    for (; q < q1; ++q) {
        const double s0 = S2[(size_t)q * nstates + jj];
#pragma unroll
        for (int t = 0; t < kZpvCT; ++t) z[t] *= fmax(0.0, fma(-c[t], s0, 1.0));
    }
#pragma unroll
    for (int t = 0; t < kZpvCT; ++t) part[slice][t][lane] = z[t];
    __syncthreads();
    const size_t rows = (size_t)nvar + 1;
    if (slice == 0 && ok) {
#pragma unroll
        for (int t = 0; t < kZpvCT; ++t) {
            double zz = part[0][t][lane];
#pragma unroll
            for (int sl = 1; sl < kZpvSlices; ++sl) zz *= part[sl][t][lane];
            if (c0 + t < nc) ZPV[(size_t)(c0 + t) * rows * nstates + j] = zz;
        }
    }
    if (ok)
        for (uint32_t b = slice; b < nvar; b += kZpvSlices) {
            const double sb = S2[(size_t)(nnv + b) * nstates + j];
#pragma unroll
            for (int t = 0; t < kZpvCT; ++t)
                if (c0 + t < nc) {
                    const double pc = c[t] * sb;
                    ZPV[((size_t)(c0 + t) * rows + 1 + b) * nstates + j] = pc > 1.0 ? 1.0 : pc;
                }
        }
}

// One workgroup per c value.
//  1. (LDS_ZPV) stage this c's Z/PV block in LDS;
//  2. lanes over transition pairs: Q_ab[m] = sum over subsets j of A&B with
//     |j| = m of Z_j * prod_{var b not in j} (B_b ? pC : 1-pC)  (subsets
//     enumerated once, accumulated per popcount in LDS);
//  3. lanes over (use, r): R[c][use][r] = sum_m Q[m] C(D-|A|, r-m).
template <bool LDS_ZPV, int NV>
__global__ __launch_bounds__(kBlock) void k_coefs(
    const double *__restrict__ ZPV, uint32_t nstates, uint32_t nvar,
    const uint32_t *__restrict__ pairA, const uint32_t *__restrict__ pairB,
    const uint32_t *__restrict__ pairOff, const uint32_t *__restrict__ items, uint32_t nitems,
    const uint32_t *__restrict__ use_pair, uint32_t nuses, uint32_t deg,
    double *__restrict__ R, size_t ldR)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const uint32_t ic = blockIdx.x;
    const size_t zsz = (size_t)(nvar + 1) * nstates;
    const double *zg = ZPV + (size_t)ic * zsz;
    const double *zpv;
    double *Qs;
    if constexpr (LDS_ZPV) {
        for (size_t i = threadIdx.x; i < zsz; i += kBlock) lds[i] = zg[i];
        zpv = lds;
        Qs = lds + zsz;
    } else {
        zpv = zg;
        Qs = lds;
    }
    __syncthreads();
    // one lane per coefficient item (pair p, popcount m): sum over the
    // C(|X|, m) subsets j of X = A&B with |j| = m (Gosper's sequence of
    // m-bit patterns over the |X| positions, deposited into X)
    for (uint32_t it = threadIdx.x; it < nitems; it += kBlock) {
        const uint32_t w = items[it];
        const uint32_t p = w >> 5, m = w & 31u;
        const uint32_t A = pairA[p], B = pairB[p], X = A & B;
        const uint32_t nX = __popc(X);
        double acc = 0.0;
        uint32_t pat = m ? ((1u << m) - 1u) : 0u;
        const uint32_t lim = 1u << nX;
        while (pat < lim) {
            uint32_t sub = 0, xs = X, bits = pat;
            while (bits) {
                const uint32_t low = xs & (0u - xs);
                if (bits & 1u) sub |= low;
                xs ^= low;
                bits >>= 1;
            }
            // branch-free: every factor load is issued up front; bits of j
            // contribute an exact 1.0
            double prod = zpv[sub];
#pragma unroll
            for (int b = 0; b < NV; ++b) {
                if ((uint32_t)b < nvar) {
                    const uint32_t bit = nvar - 1 - b;
                    const double f = zpv[(size_t)(1 + b) * nstates + sub];
                    const double g = ((B >> bit) & 1u) ? f : 1.0 - f;
                    prod *= ((sub >> bit) & 1u) ? 1.0 : g;
                }
            }
            acc += prod;
            if (pat == 0) break;
            const uint32_t t = pat | (pat - 1u);  // next pattern with the same popcount
            pat = (t + 1u) | (((~t & (0u - ~t)) - 1u) >> (__ffs(pat) ));
        }
        Qs[pairOff[p] + m] = acc;
    }
    __syncthreads();
    const uint32_t rs = deg + 1;
    double *Rc = R + (size_t)ic * ldR;
    for (uint32_t it = nuses * rs + threadIdx.x; it < (nuses + 2) * rs; it += kBlock) Rc[it] = 0.0;
    for (uint32_t it = threadIdx.x; it < nuses * rs; it += kBlock) {
        const uint32_t u = it / rs, r = it - u * rs;
        const uint32_t p = use_pair[u];
        const uint32_t A = pairA[p];
        const uint32_t nA = __popc(A), nX = __popc(A & pairB[p]);
        const uint32_t lift = deg - nA;
        const double *q = Qs + pairOff[p];
        double acc = 0.0;
        const uint32_t m0 = r > lift ? r - lift : 0;
        const uint32_t m1 = r < nX ? r : nX;
        for (uint32_t m = m0; m <= m1; ++m) acc += q[m] * c_binom[lift][r - m];
        Rc[it] = acc;
    }
}

// Dot product of one transition's coefficients (wave-uniform, SGPRs) with a
// point's weights, as two interleaved partial sums for FMA latency.
template <int RS>
__device__ __forceinline__ double tdot(const double (&rc)[RS], const double (&w)[RS])
{
    double a0 = 0.0, a1 = 0.0;
#pragma unroll
    for (int r = 0; r + 1 < RS; r += 2) {
        a0 = fma(rc[r], w[r], a0);
        a1 = fma(rc[r + 1], w[r + 1], a1);
    }
    if constexpr (RS & 1) a0 = fma(rc[RS - 1], w[RS - 1], a0);
    return a0 + a1;
}

// Coefficients are read through the constant address space: the data is
// read-only for the whole launch, so uniform reads become scalar loads even
// next to explicit s_waitcnt / sched_barrier intrinsics.
typedef const __attribute__((address_space(4))) double cdouble;

template <int RS>
__device__ __forceinline__ void tload(double (&dst)[RS], cdouble *src)
{
#pragma unroll
    for (int r = 0; r < RS; ++r) dst[r] = src[r];
}

// Forward recursion, EPL grid points per lane (e values ie, ie+256, ...), one
// c per workgroup.  Program `prog` (padded with one trailing word): one word
// per step, either a run of `count` consecutive 1x1 transitions (v0 *= P) or
// one general year (npp -> npc states, the reference's Pold*Pcur at :379).
// Inside a run the coefficient loads are software-pipelined two transitions
// ahead (R is padded by two transitions per c, so prefetches never leave it).  Q3 semantics (:368-369): start from ones over the
// year-0 states; L = sum_l v_l*prior0.
template <int NPMAX, int DEG, int EPL>
__global__ __launch_bounds__(kBlock) void k_forward(
    const double *__restrict__ R, size_t ldR, const uint32_t *__restrict__ prog, uint32_t nprog,
    uint32_t np0, double prior0, const double *__restrict__ evals, uint32_t ne,
    double *__restrict__ out, uint32_t ld_out)
{
    constexpr int RS = DEG + 1;
    const uint32_t ic = blockIdx.x;
    uint32_t ie[EPL];
    double W[EPL][RS];
    double v[EPL][NPMAX];
#pragma unroll
    for (int i = 0; i < EPL; ++i) {
        ie[i] = blockIdx.y * (kBlock * EPL) + i * kBlock + threadIdx.x;
        const double e = ie[i] < ne ? evals[ie[i]] : 0.0;
        const double x = e > 1.0 ? 1.0 : e;
        const double y = 1.0 - x;
        double yp[RS];
        yp[0] = 1.0;
#pragma unroll
        for (int r = 1; r < RS; ++r) yp[r] = yp[r - 1] * y;
        double xp = 1.0;
#pragma unroll
        for (int r = DEG; r >= 0; --r) {
            W[i][r] = xp * yp[r];
            xp *= x;
        }
#pragma unroll
        for (int k = 0; k < NPMAX; ++k) v[i][k] = (uint32_t)k < np0 ? 1.0 : 0.0;
    }

    cdouble *rp = (cdouble *)(R + (size_t)ic * ldR);  // next transition
    uint32_t op = prog[0];
    for (uint32_t pi = 0; pi < nprog; ++pi) {
        const uint32_t op_next = prog[pi + 1];
        if ((op & 1u) == 0) {
            // run of 1x1 transitions: ping-pong coefficient buffers.  Scalar
            // loads return out of order, so the only usable wait is
            // lgkmcnt(0): each half waits for its buffer, THEN issues the
            // other buffer's loads, then computes -- the loads fly under the
            // compute (sched_barrier keeps the compiler from sinking them).
            uint32_t cnt = op >> 1;
            double r0[RS], r1[RS];
            tload(r0, rp);
            for (; cnt >= 2; cnt -= 2) {
                double P[EPL];
                __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
                __builtin_amdgcn_sched_barrier(0);
                tload(r1, rp + RS);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < EPL; ++i) P[i] = tdot(r0, W[i]);
#pragma unroll
                for (int i = 0; i < EPL; ++i) v[i][0] = v[i][0] * P[i];
                __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
                __builtin_amdgcn_sched_barrier(0);
                tload(r0, rp + 2 * RS);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < EPL; ++i) P[i] = tdot(r1, W[i]);
#pragma unroll
                for (int i = 0; i < EPL; ++i) v[i][0] = v[i][0] * P[i];
                rp += 2 * RS;
            }
            if (cnt) {
#pragma unroll
                for (int i = 0; i < EPL; ++i) v[i][0] = v[i][0] * tdot(r0, W[i]);
                rp += RS;
            }
        } else {
            const uint32_t npp = (op >> 8) & 0xffu, npc = (op >> 16) & 0xffu;
            double vn[EPL][NPMAX];
#pragma unroll
            for (int l = 0; l < NPMAX; ++l) {
#pragma unroll
                for (int i = 0; i < EPL; ++i) vn[i][l] = 0.0;
                if ((uint32_t)l < npc) {
#pragma unroll
                    for (int k = 0; k < NPMAX; ++k) {
                        if ((uint32_t)k < npp) {
                            double rc[RS];
                            tload(rc, rp);
                            rp += RS;
#pragma unroll
                            for (int i = 0; i < EPL; ++i) vn[i][l] = fma(v[i][k], tdot(rc, W[i]), vn[i][l]);
                        }
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < EPL; ++i)
#pragma unroll
                for (int l = 0; l < NPMAX; ++l) v[i][l] = vn[i][l];
        }
        op = op_next;
    }
    // v beyond the last year's state count is zero: the in-order sum over all
    // NPMAX slots adds exact zeros only
#pragma unroll
    for (int i = 0; i < EPL; ++i) {
        double L = 0.0;
#pragma unroll
        for (int l = 0; l < NPMAX; ++l) L += v[i][l] * prior0;
        if (ie[i] < ne) out[(size_t)ie[i] * ld_out + ic] = log(L);
    }
}

// ---------------------------------------------------------------------------
// host side
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
    *cap = count ? count : 1;
    return MDP_OK;
}

enum { kEvBegin = 0, kEvZpv, kEvCoefs, kEvForward, kNumEv };
const char *const kKernelNames[] = {"k_zpv", "k_coefs", "k_forward"};

struct DevCtx {
    int device = 0;
    hipStream_t stream = nullptr;
    double *S = nullptr;
    uint32_t *var_cols = nullptr, *row_col = nullptr;
    uint32_t *pairA = nullptr, *pairB = nullptr, *pairOff = nullptr;
    uint32_t *use_pair = nullptr, *prog = nullptr, *items = nullptr;
    double *e = nullptr, *c = nullptr;
    size_t cap_e = 0, cap_c = 0;
    uint32_t ne = 0, nc = 0;
    double *ZPV = nullptr, *R = nullptr, *out = nullptr;
    size_t cap_zpv = 0, cap_r = 0, cap_out = 0;
    std::vector<hipEvent_t> ev;  // kNumEv events per profiled run, reused
    size_t ev_used = 0;          // event sets recorded since the last collect
};

}  // namespace

struct mdp_engine {
    uint32_t n = 0, tmax = 0, nvar = 0, nstates = 0, nextid = 0;
    uint32_t npairs = 0, nuses = 0, ncoef = 0, npmax = 1, variant = 0;
    uint32_t deg = 0;         // homogeneous transition degree D
    uint32_t maxA = 0;        // max |A| over uses
    int epl = kEPL;           // k_forward points per lane (MDP_EPL overrides: 1, 2, 4)
    bool lds_zpv = true;      // k_coefs stages Z/PV in LDS
    size_t coef_lds = 0;      // k_coefs dynamic LDS bytes
    double prior0 = 1.0;
    std::vector<uint32_t> np, pairA, pairB, pairOff, use_pair, prog, items;
    std::vector<DevCtx> devs;
    int profiling = 0;
    double last_ms[3] = {0, 0, 0};  // mean per run over the last collected runs
    int nlast = 0;
    uint64_t runs_collected = 0;
};

namespace {

constexpr int kDegBuckets[] = {2, 4, 6, 8, 12, 16, 24};

int select_variant(mdp_engine *eng)
{
    uint32_t np = 0;
    for (uint32_t b : {1u, 2u, 4u, 8u, 16u})
        if (eng->npmax <= b) { np = b; break; }
    if (!np)
        return mdp_set_error(MDP_EUNSUPPORTED,
                             "a year with %u possible states (more than 4 missing patches) "
                             "exceeds the register-resident forward kernel (max 16)", eng->npmax);
    uint32_t deg = 0;
    for (int b : kDegBuckets)
        if (eng->maxA <= (uint32_t)b) { deg = (uint32_t)b; break; }
    if (!deg) return mdp_set_error(MDP_EUNSUPPORTED, "%u occupied patches in one state (max %d)", eng->maxA, kMaxDeg);
    eng->deg = deg;
    eng->variant = np * 100 + deg;
    return MDP_OK;
}

// Host plan: distinct transition pairs (sorted by |A&B| descending for load
// balance in k_coefs), Q offsets, the per-use pair index in forward order, and
// the step program (runs of 1x1 transitions / general years).
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
    std::map<uint64_t, uint32_t> pair_index;
    std::vector<uint32_t> A0, B0, use0;
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
                    pi = (uint32_t)A0.size();
                    pair_index.emplace(key, pi);
                    A0.push_back(p->short_state[a]);
                    B0.push_back(p->short_state[b]);
                } else {
                    pi = it->second;
                }
                use0.push_back(pi);
                eng->maxA = std::max(eng->maxA, (uint32_t)__builtin_popcount(p->short_state[a]));
            }
    }
    // sort pairs by subset count (heaviest first), stable
    std::vector<uint32_t> order(A0.size());
    for (uint32_t i = 0; i < order.size(); ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
        return __builtin_popcount(A0[x] & B0[x]) > __builtin_popcount(A0[y] & B0[y]);
    });
    std::vector<uint32_t> rank(order.size());
    uint32_t off = 0;
    for (uint32_t r = 0; r < order.size(); ++r) {
        const uint32_t i = order[r];
        rank[i] = r;
        eng->pairA.push_back(A0[i]);
        eng->pairB.push_back(B0[i]);
        eng->pairOff.push_back(off);
        off += (uint32_t)__builtin_popcount(A0[i] & B0[i]) + 1u;
    }
    for (uint32_t u : use0) eng->use_pair.push_back(rank[u]);
    // k_coefs work items (pair, m), heaviest (largest C(|X|, m)) first
    {
        std::vector<std::pair<double, uint32_t>> w;
        for (uint32_t pi = 0; pi < eng->pairA.size(); ++pi) {
            const uint32_t nX = (uint32_t)__builtin_popcount(eng->pairA[pi] & eng->pairB[pi]);
            double cnk = 1.0;
            for (uint32_t m = 0; m <= nX; ++m) {
                w.emplace_back(-cnk, (pi << 5) | m);
                cnk = cnk * (double)(nX - m) / (double)(m + 1);
            }
        }
        std::stable_sort(w.begin(), w.end(),
                         [](const std::pair<double, uint32_t> &a, const std::pair<double, uint32_t> &b) {
                             return a.first < b.first;
                         });
        for (auto &x : w) eng->items.push_back(x.second);
        if (eng->pairA.size() >= (1u << 27))
            return mdp_set_error(MDP_EUNSUPPORTED, "too many transition pairs");
    }
    eng->npairs = (uint32_t)eng->pairA.size();
    eng->nuses = (uint32_t)eng->use_pair.size();
    eng->ncoef = off;
    int rc = select_variant(eng);
    if (rc) return rc;
    // step program
    for (uint32_t t = 1; t < p->tmax;) {
        if (eng->np[t - 1] == 1 && eng->np[t] == 1) {
            uint32_t cnt = 0;
            while (t < p->tmax && eng->np[t - 1] == 1 && eng->np[t] == 1) {
                ++cnt;
                ++t;
            }
            eng->prog.push_back(cnt << 1);
        } else {
            eng->prog.push_back(1u | (eng->np[t - 1] << 8) | (eng->np[t] << 16));
            ++t;
        }
    }
    eng->prog.push_back(0u);  // pad: the forward kernel reads one word ahead
    // k_coefs LDS plan
    const size_t zbytes = (size_t)(eng->nvar + 1) * eng->nstates * sizeof(double);
    const size_t qbytes = (size_t)eng->ncoef * sizeof(double);
    if (zbytes + qbytes <= kLdsBudget) {
        eng->lds_zpv = true;
        eng->coef_lds = zbytes + qbytes;
    } else if (qbytes <= kLdsBudget) {
        eng->lds_zpv = false;
        eng->coef_lds = qbytes;
    } else {
        return mdp_set_error(MDP_EUNSUPPORTED, "%u transition coefficients exceed the LDS budget",
                             eng->ncoef);
    }
    return MDP_OK;
}

int upload_binomials()  // into the current device's constant bank
{
    double h[kMaxDeg + 1][kMaxDeg + 1] = {};
    for (int a = 0; a <= kMaxDeg; ++a) {
        h[a][0] = 1.0;
        for (int b = 1; b <= a; ++b) h[a][b] = h[a][b - 1] * (double)(a - b + 1) / (double)b;
    }
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(c_binom), h, sizeof(h)));
    return MDP_OK;
}

int init_device(mdp_engine *eng, DevCtx &d, const mdp_problem *p)
{
    HIP_TRY(hipSetDevice(d.device));
    HIP_TRY(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
    int rc = upload_binomials();
    if (rc) return rc;
    std::vector<uint32_t> var(p->var_cols, p->var_cols + p->nvar), row_col;
    std::vector<uint8_t> isvar(p->n, 0);
    for (uint32_t b = 0; b < p->nvar; ++b) isvar[p->var_cols[b]] = 1;
    for (uint32_t k = 0; k < p->n; ++k)
        if (!isvar[k]) row_col.push_back(k);
    for (uint32_t b = 0; b < p->nvar; ++b) row_col.push_back(p->var_cols[b]);
    std::vector<double> M(p->M, p->M + (size_t)p->n * p->n);
    double *dM = nullptr;
    if ((rc = dev_upload(&dM, M))) return rc;
    if ((rc = dev_upload(&d.var_cols, var)) || (rc = dev_upload(&d.row_col, row_col)) ||
        (rc = dev_upload(&d.pairA, eng->pairA)) || (rc = dev_upload(&d.pairB, eng->pairB)) ||
        (rc = dev_upload(&d.pairOff, eng->pairOff)) || (rc = dev_upload(&d.use_pair, eng->use_pair)) ||
        (rc = dev_upload(&d.prog, eng->prog)) || (rc = dev_upload(&d.items, eng->items)) ||
        (rc = dev_alloc(&d.S, (size_t)p->n * eng->nstates))) {
        (void)hipFree(dM);
        return rc;
    }
    dim3 grid((eng->nstates + kBlock - 1) / kBlock, p->n);
    hipLaunchKernelGGL(k_colsum, grid, dim3(kBlock), 0, d.stream, dM, d.var_cols, d.row_col, p->n,
                       p->nvar, eng->nstates, d.S);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(d.stream));
    (void)hipFree(dM);
    if (eng->coef_lds > 64 * 1024) {
        const void *fns[] = {(const void *)k_coefs<true, 8>,   (const void *)k_coefs<true, 16>,
                             (const void *)k_coefs<true, 24>,  (const void *)k_coefs<false, 8>,
                             (const void *)k_coefs<false, 16>, (const void *)k_coefs<false, 24>};
        for (const void *fn : fns)
            HIP_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)eng->coef_lds));
    }
    return MDP_OK;
}

void free_device(DevCtx &d)
{
    (void)hipSetDevice(d.device);
    void *ptrs[] = {d.S, d.var_cols, d.row_col, d.pairA, d.pairB, d.pairOff, d.use_pair, d.prog, d.items,
                    d.e, d.c, d.ZPV, d.R, d.out};
    for (void *ptr : ptrs)
        if (ptr) (void)hipFree(ptr);
    for (hipEvent_t ev : d.ev) (void)hipEventDestroy(ev);
    if (d.stream) (void)hipStreamDestroy(d.stream);
}

// per-c coefficient stride: every forward use plus two zero transitions of
// prefetch padding
size_t ldR_of(const mdp_engine *eng) { return ((size_t)eng->nuses + 2) * (eng->deg + 1); }

int set_grid_dev(mdp_engine *eng, DevCtx &d, const double *e, uint32_t ne, const double *c,
                 uint32_t nc)
{
    HIP_TRY(hipSetDevice(d.device));
    int rc;
    if ((rc = dev_reserve(&d.e, &d.cap_e, ne)) || (rc = dev_reserve(&d.c, &d.cap_c, nc)) ||
        (rc = dev_reserve(&d.ZPV, &d.cap_zpv, (size_t)nc * (eng->nvar + 1) * eng->nstates)) ||
        (rc = dev_reserve(&d.R, &d.cap_r, (size_t)nc * ldR_of(eng))))
        return rc;
    if (ne) HIP_TRY(hipMemcpy(d.e, e, ne * sizeof(double), hipMemcpyHostToDevice));
    if (nc) HIP_TRY(hipMemcpy(d.c, c, nc * sizeof(double), hipMemcpyHostToDevice));
    d.ne = ne;
    d.nc = nc;
    return MDP_OK;
}

template <int NP, int DEG, int EPL>
void launch_fwd_epl(const mdp_engine *eng, const DevCtx &d, double *out, uint32_t ld, hipStream_t s)
{
    dim3 grid(d.nc, (d.ne + kBlock * EPL - 1) / (kBlock * EPL));
    hipLaunchKernelGGL((k_forward<NP, DEG, EPL>), grid, dim3(kBlock), 0, s, d.R, ldR_of(eng), d.prog,
                       (uint32_t)eng->prog.size() - 1, eng->np[0], eng->prior0, d.e, d.ne, out, ld);
}

template <int NP, int DEG>
void launch_fwd(const mdp_engine *eng, const DevCtx &d, double *out, uint32_t ld, hipStream_t s)
{
    if constexpr (NP <= 4 && DEG <= 8) {
        if (eng->epl == 1) return launch_fwd_epl<NP, DEG, 1>(eng, d, out, ld, s);
        if (eng->epl == 4) return launch_fwd_epl<NP, DEG, 4>(eng, d, out, ld, s);
    }
    launch_fwd_epl<NP, DEG, kEPL>(eng, d, out, ld, s);
}

template <int NP>
int launch_fwd_deg(const mdp_engine *eng, const DevCtx &d, double *out, uint32_t ld, hipStream_t s)
{
    switch (eng->deg) {
    case 2: launch_fwd<NP, 2>(eng, d, out, ld, s); break;
    case 4: launch_fwd<NP, 4>(eng, d, out, ld, s); break;
    case 6: launch_fwd<NP, 6>(eng, d, out, ld, s); break;
    case 8: launch_fwd<NP, 8>(eng, d, out, ld, s); break;
    case 12: launch_fwd<NP, 12>(eng, d, out, ld, s); break;
    case 16: launch_fwd<NP, 16>(eng, d, out, ld, s); break;
    case 24: launch_fwd<NP, 24>(eng, d, out, ld, s); break;
    default: return mdp_set_error(MDP_EUNSUPPORTED, "no forward kernel for degree %u", eng->deg);
    }
    return MDP_OK;
}

int launch_forward(const mdp_engine *eng, const DevCtx &d, double *out, uint32_t ld, hipStream_t s)
{
    int rc;
    switch (eng->variant / 100) {
    case 1: rc = launch_fwd_deg<1>(eng, d, out, ld, s); break;
    case 2: rc = launch_fwd_deg<2>(eng, d, out, ld, s); break;
    case 4: rc = launch_fwd_deg<4>(eng, d, out, ld, s); break;
    case 8: rc = launch_fwd_deg<8>(eng, d, out, ld, s); break;
    case 16: rc = launch_fwd_deg<16>(eng, d, out, ld, s); break;
    default: return mdp_set_error(MDP_EUNSUPPORTED, "no forward kernel variant %u", eng->variant);
    }
    if (rc) return rc;
    HIP_TRY(hipGetLastError());
    return MDP_OK;
}

template <bool LDS, int NV>
void launch_coefs_nv(const mdp_engine *eng, const DevCtx &d, hipStream_t s)
{
    hipLaunchKernelGGL((k_coefs<LDS, NV>), dim3(d.nc), dim3(kBlock), eng->coef_lds, s, d.ZPV,
                       eng->nstates, eng->nvar, d.pairA, d.pairB, d.pairOff, d.items,
                       (uint32_t)eng->items.size(), d.use_pair, eng->nuses, eng->deg, d.R, ldR_of(eng));
}

int launch_coefs(const mdp_engine *eng, const DevCtx &d, hipStream_t s)
{
    const uint32_t nv = eng->nvar;
    if (eng->lds_zpv) {
        if (nv <= 8) launch_coefs_nv<true, 8>(eng, d, s);
        else if (nv <= 16) launch_coefs_nv<true, 16>(eng, d, s);
        else launch_coefs_nv<true, 24>(eng, d, s);
    } else {
        if (nv <= 8) launch_coefs_nv<false, 8>(eng, d, s);
        else if (nv <= 16) launch_coefs_nv<false, 16>(eng, d, s);
        else launch_coefs_nv<false, 24>(eng, d, s);
    }
    HIP_TRY(hipGetLastError());
    return MDP_OK;
}

int run_dev(mdp_engine *eng, DevCtx &d, double *out, uint32_t ld, hipStream_t s)
{
    HIP_TRY(hipSetDevice(d.device));
    if (d.ne == 0 || d.nc == 0) return MDP_OK;
    if ((d.ne + kBlock - 1) / kBlock > 65535u || d.nc > 0x7fffffffu)
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
        dim3 grid((eng->nstates + kZpvJ - 1) / kZpvJ, (d.nc + kZpvCT - 1) / kZpvCT);
        hipLaunchKernelGGL(k_zpv, grid, dim3(kBlock), 0, s, d.S, eng->nstates, eng->n - eng->nvar,
                           eng->nvar, d.c, d.nc, d.ZPV);
        HIP_TRY(hipGetLastError());
    }
    if (prof) HIP_TRY(hipEventRecord(ev[kEvZpv], s));
    if (eng->nuses) {
        int rc = launch_coefs(eng, d, s);
        if (rc) return rc;
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
    if (const char *ev = getenv("MDP_EPL")) {
        const int v = atoi(ev);
        if (v == 1 || v == 2 || v == 4) eng->epl = v;
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
    // k_forward per point: every use is a (D+1)-term dot product (2(D+1)
    // flops) and one multiply-add into the state vector (2), plus the
    // (D+1)-term weight setup and the final prior sum.
    const double D = (double)eng->deg;
    double per_pt = (double)eng->nuses * (2.0 * (D + 1.0) + 2.0) + 3.0 * (D + 1.0) +
                    2.0 * (double)eng->npmax;
    if (flop_impl) *flop_impl = per_pt * pts;
    // SURVEY.md §8(d) F_alg (dense-in-j formulation)
    double fwd = 0;
    for (uint32_t t = 1; t < eng->tmax; ++t) fwd += (double)eng->np[t - 1] * eng->np[t];
    const double falg = 2.0 * eng->n * eng->nstates + (double)eng->nvar * eng->nstates * eng->nextid +
                        2.0 * eng->nstates * eng->npairs + 2.0 * eng->np[0] * fwd;
    if (flop_survey) *flop_survey = falg * pts;
    // compulsory bytes of k_forward: its coefficient stream once per c, the
    // e values, the output
    if (bytes_min) *bytes_min = 8.0 * ((double)nc * ldR_of(eng) + (double)ne + pts);
    return MDP_OK;
}

}  // extern "C"
