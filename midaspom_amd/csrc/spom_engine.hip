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
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "mdp_internal.h"
#include "spom_jit.h"

namespace {

constexpr int kBlock = 256;
constexpr int kZpvJ = 64;       // k_zpv: hidden states per workgroup
constexpr int kZpvSlices = 4;   // k_zpv: waves splitting the zero-column product
constexpr int kZpvCT = 2;       // k_zpv: c values per thread
constexpr int kZpvUnroll = 8;   // k_zpv: S loads in flight per lane
constexpr int kEPL = 2;         // k_forward: default grid points (e values) per lane
constexpr int kMaxDeg = 24;
constexpr int kStampSlots = 8;      // diagnostic stamps per workgroup
constexpr uint32_t kSubPart = 16;   // k_coefs: subsets per work part
constexpr uint32_t kOffBits = 22;   // coefficient offset bits in a use descriptor
constexpr uint32_t kOffMask = (1u << kOffBits) - 1u;
constexpr unsigned kWaitLgkm0 = 0xC07F;  // s_waitcnt lgkmcnt(0), other counters untouched
constexpr size_t kLdsBudget = 120 * 1024;  // dynamic LDS of k_coefs
constexpr size_t kFwdLds = 48 * 1024;      // max coefficient block staged by k_forward_lds
constexpr uint32_t kJitMaxUses = 2048;     // uses of one forward kernel; longer series run in chunks
constexpr uint32_t kJitChunkUses = 1024;   // target uses per chunk (hipRTC time grows faster than the code)
constexpr uint32_t kVldsMaxStates = 64;     // wide years the specialised kernel takes (states in LDS;
                                            // 128-state years compile to MB-sized programs)
constexpr uint32_t kVldsMaxUses = 16384;    // ... up to this many uses (hipRTC time)
constexpr size_t kJitMaxLds = 64 * 1024;   // Pc row + Q block of the direct path
constexpr size_t kJitChunkQ = kJitMaxLds / sizeof(double) - 2;  // gathered coefficients per chunk

__constant__ double c_binom[kMaxDeg + 1][kMaxDeg + 1];

// Diagnostic phase stamps (MDP_DIAG=1): wave 0 of every workgroup records
// s_memtime at phase boundaries into stamps[block][slot]; a null pointer (the
// default) skips them with one scalar branch.
#define MDP_STAMP(stamps, slot)                                                           \
    do {                                                                                  \
        if ((stamps) && threadIdx.x == 0)                                                 \
            (stamps)[(size_t)(blockIdx.x + gridDim.x * blockIdx.y) * kStampSlots + (slot)] = \
                __builtin_amdgcn_s_memtime();                                             \
    } while (0)
// wall-clock stamps (s_memrealtime, 100 MHz, chip-wide) in the last two slots
#define MDP_RSTAMP(stamps, slot)                                                          \
    do {                                                                                  \
        if ((stamps) && threadIdx.x == 0)                                                 \
            (stamps)[(size_t)(blockIdx.x + gridDim.x * blockIdx.y) * kStampSlots + (slot)] = \
                __builtin_amdgcn_s_memrealtime();                                         \
    } while (0)

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return mdp_set_error(MDP_EHIP, "%s failed: %s (%s:%d)", #expr,               \
                                 hipGetErrorString(e_), __FILE__, __LINE__);              \
    } while (0)

// Kernel timing: while an engine is profiled, every launch of a run carries
// its own start/stop events (hipExtLaunchKernel), which the runtime stamps
// from the dispatch itself -- no marker packets between the kernels, so the
// timed run is the production run and the durations agree with rocprofv3.
struct KernelEvents {
    hipEvent_t start = nullptr, stop = nullptr;
};
thread_local KernelEvents t_kev;

#define MDP_LAUNCH(kernel, grid, block, shmem, stream, ...)                                     \
    hipExtLaunchKernelGGL(kernel, grid, block, (uint32_t)(shmem), stream, t_kev.start, t_kev.stop, \
                          0u, __VA_ARGS__)

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
    const double *__restrict__ cvals, uint32_t nc, double *__restrict__ ZPV,
    unsigned long long *__restrict__ stamps)
{
    __shared__ double part[kZpvSlices][kZpvCT][kZpvJ];
    MDP_RSTAMP(stamps, 6);
    MDP_STAMP(stamps, 0);
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
        for (int t = 0; t < kZpvCT; ++t) {
            // 1 - min(1, c s), evaluated as max(0, 1 - c s) with one rounding;
            // the batch is multiplied as a tree so only one multiply per
            // batch sits on the dependency chain
            double f[kZpvUnroll];
#pragma unroll
            for (int u = 0; u < kZpvUnroll; ++u) f[u] = fmax(0.0, fma(-c[t], sv[u], 1.0));
#pragma unroll
            for (int w = 1; w < kZpvUnroll; w *= 2)
#pragma unroll
                for (int u = 0; u + w < kZpvUnroll; u += 2 * w) f[u] *= f[u + w];
            z[t] *= f[0];
        }
    }
    for (; q < q1; ++q) {
        const double s0 = S2[(size_t)q * nstates + jj];
#pragma unroll
        for (int t = 0; t < kZpvCT; ++t) z[t] *= fmax(0.0, fma(-c[t], s0, 1.0));
    }
#pragma unroll
    for (int t = 0; t < kZpvCT; ++t) part[slice][t][lane] = z[t];
    MDP_STAMP(stamps, 1);
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
    MDP_STAMP(stamps, 2);
    MDP_RSTAMP(stamps, 7);
}

// Z rows of the direct path: Zg[row][c] = prod over the always-zero columns k
// of 1 - min(1, c S[j][k]) for every needed hidden state j ("row").  Lanes run
// over c values and each wave over one row, so the S values are LDS
// broadcasts (the workgroup's rows staged once from zs[k][row]).  A broadcast
// read still returns 8 bytes per lane, so with one c per lane the kernel was
// bound by LDS return bandwidth rather than by its FMAs: each lane now
// carries kZC c values that share every read.  Same multiplication order as
// the fused forward kernel (four chains over k mod 8), so both variants give
// identical bits.
// Product of a Z row's small-column factors: exp(-c (P1 + c (P2/2 + ... +
// c P8/8))), Horner from the top (upload_qrows_tables; the fused kernel
// evaluates the same expression)
constexpr int kZTermsDev = 8;
__device__ __forceinline__ double zseries(const double (&p)[kZTermsDev], double c)
{
    double q = p[kZTermsDev - 1];
#pragma unroll
    for (int i = kZTermsDev - 2; i >= 0; --i) q = fma(q, c, p[i]);
    return exp(-(q * c));
}

constexpr uint32_t kZRows = kBlock / 64;  // rows per workgroup
constexpr uint32_t kZStage = 4;           // staging loads in flight per thread
constexpr uint32_t kZC = 2;               // c values per lane
__global__ __launch_bounds__(kBlock) void k_zrows(const double *__restrict__ cvals, uint32_t nc,
                                                  uint32_t nrows, uint32_t kmax,
                                                  const double *__restrict__ zsT, const double *__restrict__ zc,
                                                  double *__restrict__ Zg)
{
    extern __shared__ __attribute__((aligned(16))) double zl[];  // [kZRows][kmax]
    const uint32_t r0 = blockIdx.y * kZRows, nr = min(kZRows, nrows - r0);
    // the workgroup's rows are contiguous in the row-major copy zsT[row][k]:
    // coalesced loads, kZStage in flight per thread before any store
    const uint32_t nst = nr * kmax;
    for (uint32_t i0 = threadIdx.x; i0 < kZRows * kmax; i0 += kZStage * kBlock) {
        double t[kZStage];
#pragma unroll
        for (uint32_t u = 0; u < kZStage; ++u) {
            const uint32_t i = i0 + u * kBlock;
            t[u] = i < nst ? zsT[(size_t)r0 * kmax + i] : 0.0;
        }
#pragma unroll
        for (uint32_t u = 0; u < kZStage; ++u)
            if (i0 + u * kBlock < kZRows * kmax) zl[i0 + u * kBlock] = t[u];
    }
    __syncthreads();
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
    if (w >= nr) return;
    // the row's small columns: exp(-c (P1 + c (P2/2 + ...))) (upload_qrows_tables)
    double zcoef[kZTermsDev];
#pragma unroll
    for (int i = 0; i < kZTermsDev; ++i) zcoef[i] = zc[(size_t)(r0 + w) * kZTermsDev + i];
    uint32_t ic[kZC];
    double c[kZC], za[kZC], zb[kZC], zc_[kZC], zd[kZC];
#pragma unroll
    for (uint32_t x = 0; x < kZC; ++x) {
        ic[x] = blockIdx.x * (64 * kZC) + x * 64 + (threadIdx.x & 63);
        c[x] = ic[x] < nc ? cvals[ic[x]] : 0.0;
        za[x] = zb[x] = zc_[x] = zd[x] = 1.0;
    }
    const double *z = zl + w * kmax;
    auto chunk = [&](const double *sk) {
#pragma unroll
        for (uint32_t x = 0; x < kZC; ++x) {
            za[x] *= fma(-c[x], sk[0], 1.0) * fma(-c[x], sk[4], 1.0);
            zb[x] *= fma(-c[x], sk[1], 1.0) * fma(-c[x], sk[5], 1.0);
            zc_[x] *= fma(-c[x], sk[2], 1.0) * fma(-c[x], sk[6], 1.0);
            zd[x] *= fma(-c[x], sk[3], 1.0) * fma(-c[x], sk[7], 1.0);
        }
    };
    uint32_t k = 0;
    for (; k + 16 <= kmax; k += 16) {  // two chunks' reads in flight
        double sk[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) sk[u] = z[k + u];
        chunk(sk);
        chunk(sk + 8);
    }
    if (k < kmax) {  // kmax is a multiple of 8
        double sk[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) sk[u] = z[k + u];
        chunk(sk);
    }
#pragma unroll
    for (uint32_t x = 0; x < kZC; ++x) {
        double zz = (za[x] * zb[x]) * (zc_[x] * zd[x]);
        if (kmax && !(fma(-c[x], z[0], 1.0) > 0.0)) zz = 0.0;
        zz *= zseries(zcoef, c[x]);
        if (ic[x] < nc) Zg[(size_t)(r0 + w) * nc + ic[x]] = zz;
    }
}

// Transition coefficients of the direct path, one workgroup per CB (1, 2 or
// 4) consecutive c values, every hidden state j some transition needs
// ("rows", r) and every (j, b) item.  Per-c values sit interleaved in LDS in
// planes of two ([CB/2][r][2], [CB/2][item][2]) so the CB values of one row or
// item are one or two 16-byte accesses and lanes over rows / items touch
// consecutive 16-byte slots:
//  1. threads over (r, c): Z_r(c) = the row's explicit columns (zsT[row][k],
//     16 loads in flight) in k_zrows' four chains and order, the clamp test
//     against the row maximum (stored first), the small columns' series;
//  2. threads over items, all CB c values each: Pc[j][b] = Z_r prod_{var b'
//     not in j} (B_b' ? pC : 1 - pC), pC = min(1, c S[j][b']) from the row's
//     staged var-column S (-1 marks the columns of j: pC = 1.0 there);
//  3. threads over Q entries, all CB c values each: the entry's items summed
//     in CSR (ascending j) order -- written as coalesced rows for the forward
//     kernel.
// Nothing but Q leaves the workgroup.  (Round 1 kept the pressures in a
// [c][row][NV] array whose 64-byte row stride put a wave's reads on a quarter
// of the LDS banks, and ran threads over (c, item): SQ_LDS_BANK_CONFLICT was
// 3x SQ_ACTIVE_INST_LDS.)
// Canonical Q-entry sum -- k_qrows, k_wq and the fused forward kernel
// (spom_jit.cpp) all use it, so their Q rows agree bit for bit: the entry's
// items in CSR order taken in groups of kQGroup, each group summed left to
// right, and the group sums added as a pairwise tree padded with zeros to a
// power of two.  Folding the group sums into a binary counter (level l
// holds the sum of an aligned block of 2^l groups) and then folding the
// occupied levels from the lowest up gives exactly that tree; so does a
// butterfly of xor shuffles over an aligned power-of-two lane segment
// holding the sums of aligned power-of-two blocks of groups (k_qrows).
// A double from the lane DPP control CTRL names (quad_perm 0x00-0xff,
// row_mirror 0x140, row_half_mirror 0x141): no LDS, no wait
template <int CTRL>
__device__ __forceinline__ double quad_dpp(double v)
{
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

constexpr uint32_t kQGroup = 8;  // config 3: 808 lanes, one pass of k_qrows, <= 3 shuffle levels
constexpr int kQLevels = 24;
constexpr uint32_t kQLanesMax = 64;  // k_qrows: lanes per entry (a power of two, <= a wave)
constexpr int kQLevelsRows = 16;     // k_qrows: groups per lane <= 2^(kQLevelsRows - 1)

constexpr int kQrowsBlock = 1024;
constexpr uint32_t kQrowsMaxC = 4;
template <int NV, bool EXACT, int CB>  // EXACT: nvar == NV (no padded factor slots)
__global__ __launch_bounds__(kQrowsBlock) void k_qrows(
    const double *__restrict__ cvals, uint32_t nc, uint32_t nvar, uint32_t nrows,
    uint32_t kmax, const double *__restrict__ zsq, const double *__restrict__ zc, const double *__restrict__ sv,
    uint32_t nitems, const uint2 *__restrict__ items, uint32_t ncoef, const uint32_t *__restrict__ qstart,
    uint32_t nqi, const uint32_t *__restrict__ qitem, double *__restrict__ Q, uint32_t ldQ,
    unsigned long long *__restrict__ stamps, uint32_t xcd, const uint2 *__restrict__ qslot, uint32_t nslot,
    uint32_t lglmax, const uint4 *__restrict__ qlane, const uint32_t *__restrict__ islot, uint32_t npl)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    MDP_RSTAMP(stamps, 6);
    MDP_STAMP(stamps, 0);
    // phase 3's lane table does not depend on c: its first pass is loaded
    // now, its latency hidden under phases 0-2
    const uint2 sd0 = threadIdx.x < nslot ? qslot[threadIdx.x] : make_uint2(0xffffffffu, 0u);
    // nvar <= 8: the lane's group of item indices too (qlane, at least 64
    // lanes: the clamped index is in bounds)
    uint4 qa0 = make_uint4(0u, 0u, 0u, 0u), qb0 = qa0;
    if constexpr (NV == 8) {
        const uint32_t l = min(threadIdx.x, max(nslot, 1u) - 1);
        qa0 = qlane[2 * l];
        qb0 = qlane[2 * l + 1];
    }
    // XCD-aware: workgroups are dealt round-robin over the 8 XCDs, so XCD x
    // takes a contiguous eighth of the c range -- the columns the forward
    // kernel's XCD-aware order gives XCD x -- and the forward reads these Q
    // rows from its own L2
    const uint32_t nb = gridDim.x, full = nb & ~7u;
    const uint32_t lb = xcd && blockIdx.x < full ? (blockIdx.x & 7u) * (full >> 3) + (blockIdx.x >> 3) : blockIdx.x;
    const uint32_t c0 = lb * CB, ncb = min((uint32_t)CB, nc - c0);
    // per-c values in planes of two c values ([CB/2][n][2] for CB = 4): a
    // lane's 16-byte access then sits 16 bytes after its neighbour's, not 32,
    // so consecutive items / rows fill all 64 banks (no 2-way conflicts)
    constexpr uint32_t CP = CB < 2 ? CB : 2;
    auto pix = [](uint32_t n, uint32_t x, uint32_t i) -> size_t {
        return (size_t)(i / CP) * CP * n + (size_t)x * CP + i % CP;
    };
    double *Zl = lds;                                  // [CB/CP][nrows][CP]
    // per row, c and var column the pressure min(1, c S[j][b]): rows padded
    // by one double2 so rows read by one wave fall on different banks
    constexpr uint32_t PRS = CB * NV + 2;
    double *Prl = Zl + (((size_t)nrows * CB + 1) & ~(size_t)1);  // [nrows][PRS], 16-byte aligned
    // Pc per item and c in npl slots (host table islot: item -> slot);
    // slots 0-15 hold zeros, the padding phase 3's unconditional gathers
    // read past an entry's end (one per residue mod 16, so each gather group
    // can take one no other lane of it reads)
    double *Pl = Prl + (size_t)nrows * PRS;            // [CB/CP][npl][CP]
    uint32_t *Qs = (uint32_t *)(Pl + (size_t)npl * CB);  // [ncoef + 1] (nvar > 8)
    uint32_t *Qi = Qs + ncoef + 1;                     // [nqi]
    double cv[CB];  // this workgroup's c values (the last one again past the grid: never stored)
#pragma unroll
    for (int i = 0; i < CB; ++i) cv[i] = cvals[c0 + min((uint32_t)i, ncb - 1)];  // no load in a branch
    // phase 1's c value of this lane (lane q of a quad: c value q)
    const double cq = cvals[c0 + min(threadIdx.x & 3u, ncb - 1)];
    // 1. Z and pressures per row, one quad of lanes per row.  Lane q takes
    // the row's product chain q (explicit columns k = q mod 4, k_zrows' chains
    // and order) for all CB c values; the quad combines the chains as
    // (za zb)(zc zd) (exact products commute, so every lane holds the same
    // bits); lane q then finishes c value q (the clamp test against the row
    // maximum, stored first; the small columns' series) and forms var columns
    // [q NV/4, (q + 1) NV/4) of the pressures min(1, c S) of every c value
    // (the columns of j, where sv holds -1, and padded slots select a factor
    // of exactly 1.0 in phase 2 whatever is stored here).  Each row's tables
    // cross the vector cache once per workgroup: threads over (row, c) read
    // them CB times, 4x the bytes on config 3, and the cache's return rate
    // bounded the phase.
    const uint32_t kq = kmax / 4;  // chain length (kmax a multiple of 8)
    constexpr uint32_t NB = NV / 4;  // var columns per lane
    constexpr uint32_t kPre = 3;     // chain pairs loaded up front (kmax <= 24: all)
    struct RowLd {
        double2 t[kPre];  // the chain's first pairs
        double2 zq2;      // the lane's two series coefficients
        double sb[NB];    // the lane's var columns of S
    };
    auto rowload = [&](uint32_t w, RowLd &L) {
        const uint32_t q = w & 3u, r = w >> 2;
        const double2 *zr = (const double2 *)(zsq + (size_t)r * kmax + (size_t)q * kq);
#pragma unroll
        for (uint32_t u = 0; u < kPre; ++u) L.t[u] = zr[2 * u < kq ? u : 0];  // zsq padded: in bounds at kmax 0
        L.zq2 = ((const double2 *)(zc + (size_t)r * kZTermsDev))[q];
#pragma unroll
        for (uint32_t i = 0; i < NB; ++i) {
            const uint32_t b = q * NB + i;
            const double x = sv[(size_t)r * nvar + (EXACT ? b : min(b, nvar - 1))];
            L.sb[i] = (EXACT || b < nvar) ? x : HUGE_VAL;  // padded slot: pressure 1.0
        }
    };
    auto rowwork = [&](uint32_t w, const RowLd &L) {
        const uint32_t q = w & 3u, r = w >> 2;
        const double2 *zr = (const double2 *)(zsq + (size_t)r * kmax + (size_t)q * kq);
        double ch[CB];
#pragma unroll
        for (int i = 0; i < CB; ++i) ch[i] = 1.0;
        auto pair = [&](const double2 p) {
#pragma unroll
            for (int i = 0; i < CB; ++i) ch[i] *= fma(-cv[i], p.x, 1.0) * fma(-cv[i], p.y, 1.0);
        };
#pragma unroll
        for (uint32_t u = 0; u < kPre; ++u)
            if (2 * u < kq) pair(L.t[u]);
        for (uint32_t u = kPre; 2 * u < kq; u += 2) {  // longer rows (|c| > 1)
            const double2 x = zr[u], y = 2 * u + 2 < kq ? zr[u + 1] : make_double2(0.0, 0.0);
            pair(x);
            if (2 * u + 2 < kq) pair(y);
        }
        // (za zb)(zc zd) for c value q in lane q
        double c = cv[0], zz;
        if constexpr (CB == 4) {
            // reduce-scatter: the pairs (0,1), (2,3) each keep two c values
            // (lane q those = q mod 2), then (0,2), (1,3) one
            const bool b0 = q & 1u, b1 = q & 2u;
            const double s0 = b0 ? ch[0] : ch[1], s1 = b0 ? ch[2] : ch[3];
            const double k0 = (b0 ? ch[1] : ch[0]) * quad_dpp<0xB1>(s0);  // quad_perm [1,0,3,2]
            const double k1 = (b0 ? ch[3] : ch[2]) * quad_dpp<0xB1>(s1);
            zz = (b1 ? k1 : k0) * quad_dpp<0x4E>(b1 ? k0 : k1);  // quad_perm [2,3,0,1]
            c = cq;
        } else {
#pragma unroll
            for (int i = 0; i < CB; ++i) {
                ch[i] = ch[i] * quad_dpp<0xB1>(ch[i]);  // quad_perm [1,0,3,2]
                ch[i] = ch[i] * quad_dpp<0x4E>(ch[i]);  // quad_perm [2,3,0,1]
            }
            zz = ch[0];
#pragma unroll
            for (int i = 1; i < CB; ++i)
                if (q == (uint32_t)i) c = cv[i], zz = ch[i];
        }
        const double first = quad_dpp<0x00>(L.t[0].x);  // column 0, the row maximum
        if (kmax && !(fma(-c, first, 1.0) > 0.0)) zz = 0.0;
        double zq[kZTermsDev];
        zq[0] = quad_dpp<0x00>(L.zq2.x), zq[1] = quad_dpp<0x00>(L.zq2.y);
        zq[2] = quad_dpp<0x55>(L.zq2.x), zq[3] = quad_dpp<0x55>(L.zq2.y);
        zq[4] = quad_dpp<0xAA>(L.zq2.x), zq[5] = quad_dpp<0xAA>(L.zq2.y);
        zq[6] = quad_dpp<0xFF>(L.zq2.x), zq[7] = quad_dpp<0xFF>(L.zq2.y);
        zz *= zseries(zq, c);
        if (q < (uint32_t)CB) Zl[pix(nrows, r, q)] = zz;
        // min(1, c S) as the reference clamps it (:355-357): NaN stays NaN;
        // exactly 1.0 for the columns of j (sv -1) and the padded slots, so
        // that phase 2's fma(s, p, n) gives their factor 1.0 with no select
#pragma unroll
        for (int i = 0; i < CB; ++i) {
            double pr[NB];
#pragma unroll
            for (uint32_t j = 0; j < NB; ++j) {
                pr[j] = fmin(cv[i] * L.sb[j], 1.0);  // (+inf marks: 1.0, at c = 0 too -- minNum drops NaN)
            }
            double2 *pd = (double2 *)(Prl + (size_t)r * PRS + i * NV + q * NB);
#pragma unroll
            for (uint32_t j = 0; j < NB / 2; ++j) pd[j] = make_double2(pr[2 * j], pr[2 * j + 1]);
        }
    };
    // the first row's loads (index clamped: no load in a branch), then the
    // first pass of the items and Q CSR staging, both in flight at once; the
    // staging's stores wait until the row's work is done, so its latency
    // hides under phase 1
    const uint32_t nrw = nrows * 4;
    RowLd L0;
    rowload(min(threadIdx.x, nrw - 1), L0);
    constexpr uint32_t kSt = 4;
    uint2 ti[kSt];     // the items of this thread's first kSt phase-2 passes
    uint32_t si[kSt];  // and their Pc slots
    uint32_t ts[kSt], tq[kSt];
    auto stload = [&](uint32_t i0, uint2 *pi, uint32_t *ps, uint32_t *pq) {
#pragma unroll
        for (uint32_t u = 0; u < kSt; ++u) {
            const uint32_t i = i0 + u * kQrowsBlock;
            // clamped, not guarded: a guarded load sits in a branch, and the
            // row's first use then waited for every staging load too
            if (pi) {  // launched only with items
                pi[u] = items[min(i, nitems - 1)];
                si[u] = islot[min(i, nitems - 1)];
            }
            if constexpr (NV != 8) {  // nvar <= 8: phase 3 reads qlane instead
                ps[u] = qstart[min(i, ncoef)];
                pq[u] = nqi ? qitem[min(i, nqi - 1)] : 0u;
            }
        }
    };
    auto ststore = [&](uint32_t i0, const uint32_t *ps, const uint32_t *pq) {
        if constexpr (NV != 8) {
#pragma unroll
            for (uint32_t u = 0; u < kSt; ++u) {
                const uint32_t i = i0 + u * kQrowsBlock;
                if (i <= ncoef) Qs[i] = ps[u];
                if (i < nqi) Qi[i] = pq[u];
            }
        }
    };
    stload(threadIdx.x, ti, ts, tq);
    if (threadIdx.x < nrw) rowwork(threadIdx.x, L0);
    for (uint32_t w = threadIdx.x + kQrowsBlock; w < nrw; w += kQrowsBlock) {
        RowLd L;
        rowload(w, L);
        rowwork(w, L);
    }
    MDP_STAMP(stamps, 4);
    ststore(threadIdx.x, ts, tq);
    if constexpr (NV != 8) {  // a longer Q CSR (items past kSt passes are read in phase 2)
        for (uint32_t i0 = threadIdx.x + kSt * kQrowsBlock; i0 < max(ncoef + 1, nqi); i0 += kSt * kQrowsBlock) {
            uint32_t ps[kSt], pq[kSt];
            stload(i0, nullptr, ps, pq);
            ststore(i0, ps, pq);
        }
    }
    MDP_STAMP(stamps, 5);
    __syncthreads();
    MDP_STAMP(stamps, 1);
    // 2. Pc per item, its CB c values: Z times the product F of the
    // var-column factors f_b = B_b ? pC_b : 1 - pC_b (j <= B, so j's columns
    // give pC = 1.0, a factor of exactly 1.0), in the pairwise tree over NV
    // slots -- the fused kernel's tree over nvar (padded slots are 1.0).  A
    // factor is |n_b - pC_b| with n_b = 1.0 where B_b is clear, 0.0 where set:
    // the same bits as the fused kernel's fma(s_b, pC_b, n_b), s_b = -1 / +1
    // (1 - p rounded once; |0 - p| = p exactly), with the bit converted once
    // per item and the abs folded into the tree's first products.  (Building
    // s_b and n_b as doubles cost 5 integer instructions a slot, a quarter-rate
    // multiply among them: phase 2 is bound by VALU issue.)
    // the first kSt passes' items are still in this thread's staging
    // registers (pass u's item is the one it loaded as ti[u])
    auto pcitem = [&](uint32_t sl, const uint2 t) {
        const uint32_t r = (t.x >> 24) | ((t.y >> 24) << 8), nB = ~t.x;
        double nb[NV];
#pragma unroll
        for (int b = 0; b < NV; ++b) {
            const uint32_t bit = EXACT ? (uint32_t)(NV - 1 - b) : nvar - 1 - (uint32_t)b;  // wraps past nvar
            const uint32_t nbit = !EXACT && (uint32_t)b >= nvar ? 0u : (nB >> bit) & 1u;
            nb[b] = (double)nbit;
        }
        double zr[CB], pc[CB];
#pragma unroll
        for (int i = 0; i < CB; ++i) zr[i] = Zl[pix(nrows, r, i)];
#pragma unroll
        for (int i = 0; i < CB; ++i) {
            double f[NV];
            const double2 *ps = (const double2 *)(Prl + (size_t)r * PRS + i * NV);
#pragma unroll
            for (int b = 0; b < NV / 2; ++b) {
                const double2 p2 = ps[b];
                f[2 * b] = fabs(nb[2 * b] - p2.x) * fabs(nb[2 * b + 1] - p2.y);
            }
#pragma unroll
            for (int sh = 2; sh < NV; sh *= 2)
#pragma unroll
                for (int b = 0; b + sh < NV; b += 2 * sh) f[b] *= f[b + sh];
            pc[i] = zr[i] * f[0];
        }
#pragma unroll
        for (int i = 0; i < CB; ++i) Pl[pix(npl, sl, i)] = pc[i];
    };
#pragma unroll
    for (uint32_t u = 0; u < kSt; ++u)
        if (threadIdx.x + u * kQrowsBlock < nitems) pcitem(si[u], ti[u]);
    for (uint32_t it = threadIdx.x + kSt * kQrowsBlock; it < nitems; it += kQrowsBlock) pcitem(islot[it], items[it]);
    if (threadIdx.x < 16 * CB) Pl[pix(npl, threadIdx.x / CB, threadIdx.x % CB)] = 0.0;
    __syncthreads();
    MDP_STAMP(stamps, 2);
    // 3. Q rows in the canonical order.  Each entry owns an aligned
    // power-of-two segment of L <= kQLanesMax lanes of one wave (host table
    // qslot: {entry, lane in entry | log2 L << 8 | log2 G << 12}, nslot a
    // multiple of 64); a lane sums its 2^G consecutive groups for the CB c
    // values (binary counter), then the segment adds the lanes' sums by a
    // butterfly of xor shuffles, and its first lane stores the entry.  The
    // chain per lane is a few gathers and log2 L shuffles instead of the
    // entry's whole item list (35 on config 3).
    if constexpr (NV == 8) {
        // nvar <= 8: one group per lane (an entry has at most C(8,4) = 70
        // items, 9 groups), its items' Pc slots in registers since the kernel
        // began (qlane: the group padded with a zero slot, x + 0.0 = x for
        // these non-negative, NaN or infinite values), so the gathers follow
        // the barrier directly; the slots are coloured on the host so that
        // each gather group's 16-byte slots fall on distinct banks.  The butterfly runs on DPP: after
        // level l every lane of an aligned 2^(l+1) block holds the same bits
        // (the sums commute exactly), so any lane of the partner block will
        // do -- quad_perm for levels 0-1, row_half_mirror and row_mirror for
        // levels 2-3, an xor shuffle beyond.
        for (uint32_t s0 = 0; s0 < nslot; s0 += kQrowsBlock) {
            const uint32_t sl = s0 + threadIdx.x;
            uint2 sd = sd0;
            uint4 qa = qa0, qb = qb0;
            if (s0 != 0) {
                const uint32_t l = min(sl, nslot - 1);
                sd = sl < nslot ? qslot[l] : make_uint2(0xffffffffu, 0u);
                qa = qlane[2 * l];
                qb = qlane[2 * l + 1];
            }
            const uint32_t q = sd.x, le = sd.y & 0xffu, lgL = (sd.y >> 8) & 0xfu;
            const uint32_t itm[kQGroup] = {qa.x, qa.y, qa.z, qa.w, qb.x, qb.y, qb.z, qb.w};
            double a[CB];
#pragma unroll
            for (int i = 0; i < CB; ++i) {
                double x = Pl[pix(npl, itm[0], i)];
#pragma unroll
                for (uint32_t u = 1; u < kQGroup; ++u) x = x + Pl[pix(npl, itm[u], i)];
                a[i] = x;
            }
            auto level = [&](uint32_t lv, auto part) {
                if (lv >= lglmax) return;  // uniform
#pragma unroll
                for (int i = 0; i < CB; ++i) {
                    const double o = part(a[i]), t = a[i] + o;
                    a[i] = lv < lgL ? t : a[i];  // a select, not a branch per value
                }
            };
            level(0, [](double v) { return quad_dpp<0xB1>(v); });   // quad_perm [1,0,3,2]
            level(1, [](double v) { return quad_dpp<0x4E>(v); });   // quad_perm [2,3,0,1]
            level(2, [](double v) { return quad_dpp<0x141>(v); });  // row_half_mirror
            level(3, [](double v) { return quad_dpp<0x140>(v); });  // row_mirror
            for (uint32_t lv = 4; lv < lglmax; ++lv)
#pragma unroll
                for (int i = 0; i < CB; ++i) {
                    const double o = __shfl_xor(a[i], 1 << lv);
                    if (lv < lgL) a[i] = a[i] + o;
                }
            if (q < ldQ && le == 0)
#pragma unroll
                for (int i = 0; i < CB; ++i)
                    if ((uint32_t)i < ncb) Q[(size_t)(c0 + i) * ldQ + q] = a[i];
        }
    } else
    for (uint32_t s0 = 0; s0 < nslot; s0 += kQrowsBlock) {
        const uint32_t sl = s0 + threadIdx.x;
        const uint2 sd = s0 == 0 ? sd0 : sl < nslot ? qslot[sl] : make_uint2(0xffffffffu, 0u);
        const uint32_t q = sd.x, le = sd.y & 0xffu, lgL = (sd.y >> 8) & 0xfu, lgG = (sd.y >> 12) & 0xfu;
        double a[CB];
#pragma unroll
        for (int i = 0; i < CB; ++i) a[i] = 0.0;
        if (q < ncoef) {
            const uint32_t i0 = Qs[q], i1 = Qs[q + 1];
            // this lane's group sums: one group (nvar <= 8: an entry has at
            // most C(8,4) = 70 items, 18 groups, so its segment takes them
            // one per lane), else 2^G consecutive groups in a binary counter
            auto group = [&](uint32_t j0, double *sg) {
#pragma unroll
                for (int i = 0; i < CB; ++i) sg[i] = 0.0;
                if (j0 >= i1) return;
                // items past the entry read the zero slot: x + (+0.0) = x for
                // these non-negative (or NaN / inf) values, so the sums are the
                // canonical order's bits without a select per item
                uint32_t itm[kQGroup];
#pragma unroll
                for (uint32_t u = 0; u < kQGroup; ++u) {
                    const uint32_t t_ = Qi[j0 + u < i1 ? j0 + u : j0];
                    itm[u] = j0 + u < i1 ? t_ + 16 : 0u;  // slots (nvar > 8: item + 16)
                }
#pragma unroll
                for (int i = 0; i < CB; ++i) {
                    double x = Pl[pix(npl, itm[0], i)];
#pragma unroll
                    for (uint32_t u = 1; u < kQGroup; ++u) x = x + Pl[pix(npl, itm[u], i)];
                    sg[i] = x;
                }
            };
            if constexpr (NV == 8) {
                group(i0 + le * kQGroup, a);
            } else {
                double lev[CB][kQLevelsRows];
                const uint32_t ng = 1u << lgG;
                for (uint32_t g = 0; g < ng; ++g) {
                    double sg[CB];
                    group(i0 + ((le << lgG) + g) * kQGroup, sg);
#pragma unroll
                    for (int l = 0; l < kQLevelsRows; ++l) {
                        if ((g >> l) & 1u) {
#pragma unroll
                            for (int i = 0; i < CB; ++i) sg[i] = lev[i][l] + sg[i];
                        } else {
#pragma unroll
                            for (int i = 0; i < CB; ++i) lev[i][l] = sg[i];
                            break;
                        }
                    }
                    if (g + 1 == ng)  // 2^G groups: the counter holds one block
#pragma unroll
                        for (int i = 0; i < CB; ++i) a[i] = sg[i];
                }
            }
        }
        // every lane of the wave takes part in every shuffle; a lane adds
        // only the levels inside its entry's segment
        for (uint32_t lv = 0; lv < lglmax; ++lv)  // lglmax: the widest segment's levels (uniform)
#pragma unroll
            for (int i = 0; i < CB; ++i) {
                const double o = __shfl_xor(a[i], 1 << lv);
                if (lv < lgL) a[i] = a[i] + o;
            }
        if (q < ldQ && le == 0)
#pragma unroll
            for (int i = 0; i < CB; ++i)
                if ((uint32_t)i < ncb) Q[(size_t)(c0 + i) * ldQ + q] = a[i];
    }
    MDP_STAMP(stamps, 3);
    MDP_RSTAMP(stamps, 7);
}

// One workgroup per c value.
//  1. stage this c's Z/PV block (LDS_ZPV) and the binomial table in LDS;
//  2. subset products: lane per part (pair p, 16 consecutive subset indexes k
//     of X = A&B): j = deposit(k, X), Pc[j][b] = Z_j prod_{var b not in j}
//     (B_b ? pC : 1-pC) accumulated into the part's per-|j| partial sums;
//  3. Q_ab[m] = sum of the pair's part partials, in part order;
//  4. lane per forward use: R[c][use][r] = sum_m Q[m] C(D-|A|, r-m), padded
//     to the even stride RSP, plus two zero transitions of prefetch padding.
// Every reduction runs in a fixed order, so results are deterministic.
template <bool LDS_ZPV, bool LDS_PART, int NV>
__global__ __launch_bounds__(kBlock) void k_coefs(
    const double *__restrict__ ZPV, uint32_t nstates, uint32_t nvar,
    const uint32_t *__restrict__ pairA, const uint32_t *__restrict__ pairB,
    const uint32_t *__restrict__ pairOff, const uint32_t *__restrict__ pairPart0,
    uint32_t npairs, const uint32_t *__restrict__ partP, const uint32_t *__restrict__ partK0,
    uint32_t nparts, uint32_t ncoef, const uint32_t *__restrict__ udesc, uint32_t nuses,
    uint32_t deg, double *__restrict__ R, size_t ldR, double *__restrict__ gpart,
    unsigned long long *__restrict__ stamps)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    MDP_RSTAMP(stamps, 6);
    MDP_STAMP(stamps, 0);
    const uint32_t ic = blockIdx.x;
    const size_t zsz = (size_t)(nvar + 1) * nstates;
    const double *zg = ZPV + (size_t)ic * zsz;
    double *base = lds;
    const double *zpv = zg;
    if constexpr (LDS_ZPV) {
        for (size_t i0 = 0; i0 < zsz; i0 += 8 * kBlock) {  // 8 loads in flight per lane
            double t[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const size_t i = i0 + u * kBlock + threadIdx.x;
                if (i < zsz) t[u] = zg[i];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const size_t i = i0 + u * kBlock + threadIdx.x;
                if (i < zsz) lds[i] = t[u];
            }
        }
        zpv = lds;
        base = lds + zsz;
    }
    const uint32_t pw = nvar + 1;  // partial sums per part
    double *partial = LDS_PART ? base : gpart + (size_t)ic * nparts * pw;
    double *Qs = LDS_PART ? base + (size_t)nparts * pw : base;
    double *binom = Qs + ncoef;  // [kMaxDeg+1][kMaxDeg+1]
    for (uint32_t i = threadIdx.x; i < (kMaxDeg + 1) * (kMaxDeg + 1); i += kBlock)
        binom[i] = c_binom[i / (kMaxDeg + 1)][i % (kMaxDeg + 1)];
    __syncthreads();
    MDP_STAMP(stamps, 1);

    for (uint32_t it = threadIdx.x; it < nparts; it += kBlock) {
        const uint32_t p = partP[it], k0 = partK0[it];
        const uint32_t B = pairB[p], X = pairA[p] & B;
        const uint32_t nX = __popc(X);
        double *acc = partial + (size_t)it * pw;
        for (uint32_t m = 0; m <= nX; ++m) acc[m] = 0.0;
        const uint32_t k1 = min(k0 + kSubPart, 1u << nX);
        for (uint32_t k = k0; k < k1; ++k) {
            // deposit the bits of k into the positions of X (once X's bits are
            // used up `low` is 0 and the remaining steps are no-ops)
            uint32_t sub = 0, xs = X;
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                const uint32_t low = xs & (0u - xs);
                sub |= ((k >> i) & 1u) ? low : 0u;
                xs ^= low;
            }
            // branch-free: every factor load is issued up front (rows past
            // nvar are clamped and neutralised); bits of j contribute 1.0
            double f[NV];
#pragma unroll
            for (int b = 0; b < NV; ++b) {
                const uint32_t row = (uint32_t)b < nvar ? (uint32_t)b : nvar - 1;
                f[b] = zpv[(size_t)(1 + row) * nstates + sub];
            }
            double prod = zpv[sub];
#pragma unroll
            for (int b = 0; b < NV; ++b) {
                const uint32_t bit = nvar - 1 - (uint32_t)b;  // wraps past nvar: masked below
                const double g = ((B >> bit) & 1u) ? f[b] : 1.0 - f[b];
                const bool skip = (uint32_t)b >= nvar || ((sub >> bit) & 1u);
                prod *= skip ? 1.0 : g;
            }
            acc[__popc(k)] += prod;
        }
    }
    __syncthreads();
    MDP_STAMP(stamps, 2);
    for (uint32_t p = threadIdx.x; p < npairs; p += kBlock) {
        const uint32_t nX = __popc(pairA[p] & pairB[p]);
        const uint32_t q0 = pairPart0[p], q1 = pairPart0[p + 1];
        double *q = Qs + pairOff[p];
        for (uint32_t m = 0; m <= nX; ++m) {
            double a = 0.0;
            for (uint32_t t = q0; t < q1; ++t) a += partial[(size_t)t * pw + m];
            q[m] = a;
        }
    }
    __syncthreads();
    MDP_STAMP(stamps, 3);
    const uint32_t rsp = (deg + 2) & ~1u;
    double *Rc = R + (size_t)ic * ldR;
    for (uint32_t it = nuses * rsp + threadIdx.x; it < (nuses + 2) * rsp; it += kBlock) Rc[it] = 0.0;
    for (uint32_t u = threadIdx.x; u < nuses; u += kBlock) {
        const uint32_t d = udesc[u];
        const double *q = Qs + (d & kOffMask);
        const uint32_t nX = (d >> kOffBits) & 31u, nA = d >> 27;
        const uint32_t lift = deg - nA;
        const double *bl = binom + lift * (kMaxDeg + 1);
        double *dst = Rc + (size_t)u * rsp;
        for (uint32_t r = 0; r < rsp; ++r) {
            double a = 0.0;
            if (r <= deg) {
                const uint32_t m0 = r > lift ? r - lift : 0;
                const uint32_t m1 = r < nX ? r : nX;
                for (uint32_t m = m0; m <= m1; ++m) a += q[m] * bl[r - m];
            }
            dst[r] = a;
        }
    }
    MDP_STAMP(stamps, 4);
    MDP_RSTAMP(stamps, 7);
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

// RS coefficients from a 16-byte aligned LDS block (ds_read_b128 pairs).
template <int RS>
__device__ __forceinline__ void tload_l(double (&dst)[RS], const double *src)
{
    const double2 *s2 = (const double2 *)src;
#pragma unroll
    for (int r = 0; r + 1 < RS; r += 2) {
        const double2 q = s2[r / 2];
        dst[r] = q.x;
        dst[r + 1] = q.y;
    }
    if constexpr (RS & 1) dst[RS - 1] = src[RS - 1];
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
    double *__restrict__ out, uint32_t ld_out, uint32_t out_cs)
{
    constexpr int RS = DEG + 1;
    constexpr int RSP = (DEG + 2) & ~1;  // per-transition stride in R
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
                tload(r1, rp + RSP);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < EPL; ++i) P[i] = tdot(r0, W[i]);
#pragma unroll
                for (int i = 0; i < EPL; ++i) v[i][0] = v[i][0] * P[i];
                __builtin_amdgcn_s_waitcnt(kWaitLgkm0);
                __builtin_amdgcn_sched_barrier(0);
                tload(r0, rp + 2 * RSP);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < EPL; ++i) P[i] = tdot(r1, W[i]);
#pragma unroll
                for (int i = 0; i < EPL; ++i) v[i][0] = v[i][0] * P[i];
                rp += 2 * RSP;
            }
            if (cnt) {
#pragma unroll
                for (int i = 0; i < EPL; ++i) v[i][0] = v[i][0] * tdot(r0, W[i]);
                rp += RSP;
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
                            rp += RSP;
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
        if (ie[i] < ne) out[(size_t)ie[i] * ld_out + (size_t)ic * out_cs] = log(L);
    }
}



// Same recursion with the workgroup's whole coefficient block (and the step
// program) staged in LDS by wide coalesced loads: transitions are then read
// with in-order ds_read_b128 broadcasts instead of scalar loads, so there is no
// scalar-cache miss on the critical path.  Used when the block fits kFwdLds.
template <int NPMAX, int DEG, int EPL>
__global__ __launch_bounds__(kBlock) void k_forward_lds(
    const double *__restrict__ R, size_t ldR, const uint32_t *__restrict__ prog, uint32_t nprog,
    uint32_t np0, double prior0, const double *__restrict__ evals, uint32_t ne,
    double *__restrict__ out, uint32_t ld_out, uint32_t out_cs, unsigned long long *__restrict__ stamps)
{
    constexpr int RS = DEG + 1;
    constexpr int RSP = (DEG + 2) & ~1;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    MDP_RSTAMP(stamps, 6);
    MDP_STAMP(stamps, 0);
    double *Rl = lds;
    uint32_t *pl = (uint32_t *)(lds + ldR);
    const uint32_t ic = blockIdx.x;
    {
        const double2 *src = (const double2 *)(R + (size_t)ic * ldR);
        double2 *dst = (double2 *)Rl;
        const uint32_t n2 = (uint32_t)(ldR / 2);
        for (uint32_t i0 = threadIdx.x; i0 < n2; i0 += 4 * kBlock) {  // 4 loads in flight per lane
            const uint32_t i1 = i0 + kBlock, i2 = i0 + 2 * kBlock, i3 = i0 + 3 * kBlock;
            const double2 t0 = src[i0];
            const double2 t1 = src[i1 < n2 ? i1 : i0];
            const double2 t2 = src[i2 < n2 ? i2 : i0];
            const double2 t3 = src[i3 < n2 ? i3 : i0];
            dst[i0] = t0;
            if (i1 < n2) dst[i1] = t1;
            if (i2 < n2) dst[i2] = t2;
            if (i3 < n2) dst[i3] = t3;
        }
        for (uint32_t i = threadIdx.x; i <= nprog; i += kBlock) pl[i] = prog[i];
    }
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
    __syncthreads();
    MDP_STAMP(stamps, 1);
    const double *rp = Rl;
    unsigned long long cyc_run = 0, cyc_gen = 0;  // diagnostic accounting only
    for (uint32_t pi = 0; pi < nprog; ++pi) {
        const uint32_t op = pl[pi];
        const unsigned long long t_op = stamps ? __builtin_amdgcn_s_memtime() : 0ull;
        if ((op & 1u) == 0) {
            uint32_t cnt = op >> 1;
            for (; cnt >= 2; cnt -= 2, rp += 2 * RSP) {
                double ra[RS], rb[RS];
                tload_l(ra, rp);
                tload_l(rb, rp + RSP);
#pragma unroll
                for (int i = 0; i < EPL; ++i) v[i][0] = v[i][0] * tdot(ra, W[i]);
#pragma unroll
                for (int i = 0; i < EPL; ++i) v[i][0] = v[i][0] * tdot(rb, W[i]);
            }
            if (cnt) {
                double ra[RS];
                tload_l(ra, rp);
                rp += RSP;
#pragma unroll
                for (int i = 0; i < EPL; ++i) v[i][0] = v[i][0] * tdot(ra, W[i]);
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
                            tload_l(rc, rp);
                            rp += RSP;
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
        if (stamps) {
            const unsigned long long dt = __builtin_amdgcn_s_memtime() - t_op;
            if (op & 1u) cyc_gen += dt;
            else cyc_run += dt;
        }
    }
    if (stamps && threadIdx.x == 0) {
        stamps[(size_t)(blockIdx.x + gridDim.x * blockIdx.y) * kStampSlots + 3] = cyc_run;
        stamps[(size_t)(blockIdx.x + gridDim.x * blockIdx.y) * kStampSlots + 4] = cyc_gen;
    }
#pragma unroll
    for (int i = 0; i < EPL; ++i) {
        double L = 0.0;
#pragma unroll
        for (int l = 0; l < NPMAX; ++l) L += v[i][l] * prior0;
        if (ie[i] < ne) out[(size_t)ie[i] * ld_out + (size_t)ic * out_cs] = log(L);
    }
    MDP_STAMP(stamps, 2);
    MDP_RSTAMP(stamps, 7);
}

// ---------------------------------------------------------------------------
// wide path: years with more observed states than the register-resident
// forward kernels hold (npmax > 16, i.e. more than 4 missing patches in one
// year; main_MIDASPOM.c:225-251 expands 2^k states for any k and propagates
// them with dgemm, :371-384).  Same direct-path algebra (Q per (X, B) group,
// DESIGN.md §3), but nothing has to fit a workgroup: the item factors and Q
// rows go through HBM/L2, and the state vectors live in an HBM scratch laid
// out [state][point] so every lane's access is coalesced.
// ---------------------------------------------------------------------------

// Pg[cl * ldp + it] = Pc[j][B] of item `it` at c = cvals[c0 + cl] (ldp: nitems,
// or nitems + 1 for k_fwd_hs, whose rows end in a zero slot): Z_row(c) times the
// var-column factors f_b = B_b ? pC_b : 1 - pC_b, pC_b = min(1, c S[j][b])
// (1.0 for the columns of j, marked -1 in sv), combined in k_qrows' pairwise
// tree over NV slots -- the same bits k_qrows produces.
template <int NV>
__global__ __launch_bounds__(kBlock) void k_witems(const double *__restrict__ cvals, uint32_t nc, uint32_t c0,
                                                   uint32_t nvar, const double *__restrict__ Zg,
                                                   const double *__restrict__ sv, uint32_t nitems,
                                                   const uint2 *__restrict__ items, double *__restrict__ Pg,
                                                   uint32_t ldp)
{
    const uint32_t it = blockIdx.x * kBlock + threadIdx.x, cl = blockIdx.y;
    if (it >= nitems) return;
    const double c = cvals[c0 + cl];
    const uint2 t = items[it];
    const uint32_t r = (t.x >> 24) | ((t.y >> 24) << 8), nB = ~t.x;
    double f[NV];
#pragma unroll
    for (int b = 0; b < NV; ++b) {
        const double sb = (uint32_t)b < nvar ? sv[(size_t)r * nvar + b] : HUGE_VAL;
        const double p = fmin(c * sb, 1.0);  // (k_qrows' form: +inf marks give 1.0)
        const uint32_t nbit = (uint32_t)b < nvar ? (nB >> (nvar - 1 - (uint32_t)b)) & 1u : 0u;
        f[b] = (double)nbit - p;  // |n - p|: k_qrows' fold
    }
#pragma unroll
    for (int b = 0; b < NV; b += 2) f[b] = fabs(f[b]) * fabs(f[b + 1]);
#pragma unroll
    for (int sh = 2; sh < NV; sh *= 2)
#pragma unroll
        for (int b = 0; b + sh < NV; b += 2 * sh) f[b] *= f[b + sh];
    Pg[(size_t)cl * ldp + it] = Zg[(size_t)r * nc + c0 + cl] * f[0];
}

// Q[c0 + cl][q] = the q-th entry's items summed in CSR (ascending j) order,
// as k_qrows sums them; zero in the padding slots up to ldQ.
__global__ __launch_bounds__(kBlock) void k_wq(uint32_t c0, uint32_t nitems, const double *__restrict__ Pg,
                                               uint32_t ncoef, const uint32_t *__restrict__ qstart,
                                               const uint32_t *__restrict__ qitem, double *__restrict__ Q,
                                               uint32_t ldQ)
{
    const uint32_t q = blockIdx.x * kBlock + threadIdx.x, cl = blockIdx.y;
    if (q >= ldQ) return;
    double a = 0.0;
    if (q < ncoef) {  // the canonical order (kQGroup): groups, binary counter, fold
        const double *pl = Pg + (size_t)cl * nitems;
        const uint32_t i0 = qstart[q], i1 = qstart[q + 1];
        double lev[kQLevels];
        uint32_t g = 0;
        for (uint32_t i = i0; i < i1; i += kQGroup, ++g) {
            double sg = pl[qitem[i]];
            for (uint32_t u = 1; u < kQGroup && i + u < i1; ++u) sg = sg + pl[qitem[i + u]];
#pragma unroll
            for (int l = 0; l < kQLevels; ++l) {
                if ((g >> l) & 1u) {
                    sg = lev[l] + sg;
                } else {
                    lev[l] = sg;
                    break;
                }
            }
        }
        bool have = false;
#pragma unroll
        for (int l = 0; l < kQLevels; ++l)
            if ((g >> l) & 1u) {
                a = have ? lev[l] + a : lev[l];
                have = true;
            }
    }
    Q[(size_t)(c0 + cl) * ldQ + q] = a;
}

// Wide years on the matrix cores (FP64 MFMA, v_mfma_f64_16x16x4_f64).  For
// one column c and a block of PTS points, year t's new state vector is
//     n[p][l] = sum_(k, m) W[p][(k, m)] C[(k, m)][l],
//     W[p][(k, m)] = v[p][k] x_p^(|A_k| - m) y_p^m,   C[(k, m)][l] = Q_kl[m]
// (0 past the transition's nX): the transition P[k][l] = sum_m Q_kl[m]
// x^(|A|-m) y^m of the wide kernels (direct weights, as k_fwd_wide), summed
// over K = every source's (k, m <= |A_k|) -- one GEMM per year of M = the
// points, N = the new states, K = sum_k (|A_k| + 1), on the matrix cores with
// the states of the block's points in LDS.  Each MFMA computes the transposed
// tile n^T = C^T W^T (A operand: the gathered C values, states x K; B: the
// W values, K x points), so a lane's accumulators are 4 states of one point
// and the year's stores are rows of 16 consecutive points (conflict-free).
// C's fragments are gathered from the column's Q row: a lane's K entry (k, m,
// the LDS rows of v_k, x^(|A_k|-m) and y^m) names the transition descriptor
// (k, l) (host table, c-independent: the Q-row offset of the transition's
// coefficients and its nX), and m <= nX picks the slot, else the zero slot.
// 16 waves, one work item each per year: (column tile, every row tile, slice
// of the year's K chunks) -- with S = min(16 / ncol, room, nch / 2) slices, so
// that up to 16 waves are busy in a year of any size.  Slice 1 leaves its
// partial products in the year's own destination rows, later slices in the
// state buffer's rows past the year's column tiles; slice 0 adds them in
// slice order (deterministic).  Each lane's K entries run three chunks ahead
// in a ring of four register slots (loaded once, straight from the table in
// HBM: staging three years of them in LDS was 1-5 % slower), the
// transition descriptors two and the C gathers one; the loop body is
// unrolled four times so the slots are fixed.  The products sum in another
// order than k_fwd_wide's (positive terms: ~1e-15 relative).
constexpr uint32_t kMmaThreads = 1024;  // 16 waves
constexpr uint32_t kMmaU = 2;           // K steps (of 4) per pipeline chunk: years padded to 8 entries
constexpr uint32_t kMmaDummy = 1u << 21; // K-entry field of the descriptor row k (bits 21-28)
// the kernel's shape for NPM states a year (padded to 16): points per block,
// state buffer rows (>= 128, for the slices' partial sums), power-table row
// stride (rows r and r + 1 on different LDS bank halves)
constexpr uint32_t mma_pts(uint32_t npm) { return npm > 128 ? 32u : 64u; }
constexpr uint32_t mma_rows(uint32_t npm) { return npm > 128 ? npm : 128u; }
constexpr uint32_t mma_ps(uint32_t npm) { return mma_pts(npm) + 16u; }
typedef double mdp_d4 __attribute__((ext_vector_type(4)));
template <int NPM>  // states per year, padded (64, 128 or 256)
__global__ __launch_bounds__(kMmaThreads) void k_fwd_mma(
    const double *__restrict__ Q, uint32_t ldQ, const uint32_t *__restrict__ np, const uint2 *__restrict__ kt,
    const uint32_t *__restrict__ kbase, const uint32_t *__restrict__ desc, const uint32_t *__restrict__ dbase,
    const uint2 *__restrict__ wplan, uint32_t tmax, double prior0, const double *__restrict__ evals, uint32_t ne,
    uint32_t c0, uint32_t maxA, uint32_t ktmax, uint32_t zslot, double *__restrict__ out, uint32_t ld_out,
    uint32_t out_cs)
{
    constexpr uint32_t PTS = mma_pts(NPM), ROWS = mma_rows(NPM), PS = mma_ps(NPM), RT = PTS / 16;
    static_assert(NPM <= (int)ROWS && NPM <= 256, "state rows");
    extern __shared__ __attribute__((aligned(16))) double mlds[];
    double *Va = mlds, *Vb = mlds + (size_t)ROWS * PTS;  // [state][point]
    double *xp = Vb + (size_t)ROWS * PTS, *yp = xp + (size_t)(maxA + 1) * PS;  // [r][point]
    const uint32_t lane = threadIdx.x & 63u, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform
    const uint32_t p0 = blockIdx.x * PTS, ic = c0 + blockIdx.y;
    if (threadIdx.x < PTS) {
        const uint32_t ie = p0 + threadIdx.x;
        const double e = ie < ne ? evals[ie] : 0.0;
        const double x = e > 1.0 ? 1.0 : e, y = 1.0 - x;
        double a = 1.0, b = 1.0;
        for (uint32_t r = 0; r <= maxA; ++r) {
            xp[r * PS + threadIdx.x] = a;
            yp[r * PS + threadIdx.x] = b;
            a *= x;
            b *= y;
        }
    }
    const uint32_t np0 = np[0];
    for (uint32_t i = threadIdx.x; i < (uint32_t)NPM * PTS; i += kMmaThreads) Va[i] = i / PTS < np0 ? 1.0 : 0.0;
    __syncthreads();
    const double *q = Q + (size_t)ic * ldQ;
    const uint32_t kk = lane >> 4, col = lane & 15u;
    // this wave's work item of year t
    struct Item {
        uint32_t npc, npcp, nch, nit, S, item, ks, cb, ce, sh, lc4;
        bool active;
        const uint2 *kl;
        const uint32_t *dt;
    };
    // (the host's work split, mma_wave_plan: one scalar load, no divisions)
    auto plan = [&](uint32_t t) {
        Item it;
        it.npc = np[t];
        const uint32_t ncol = (it.npc + 15) / 16;
        it.npcp = ncol * 16;
        it.nch = (kbase[t + 1] - kbase[t]) / (4 * kMmaU);
        it.nit = ncol;
        const uint2 wp = wplan[t * 16 + wv];
        it.cb = wp.x & 0xffffu;
        it.ce = wp.x >> 16;
        it.item = wp.y & 0xffu;
        it.ks = (wp.y >> 8) & 0xffu;
        it.S = (wp.y >> 16) & 0xffu;
        it.active = (wp.y >> 24) != 0u;
        // descriptor rows [k][2^sh >= npcp] (row npp: the padded entries')
        it.sh = 32u - (uint32_t)__builtin_clz(it.npcp - 1u);
        it.lc4 = (it.item * 16 + col) << 2;
        it.kl = kt + __builtin_amdgcn_readfirstlane(kbase[t]);
        it.dt = desc + __builtin_amdgcn_readfirstlane(dbase[t]);
        return it;
    };
    // the lane's K entry (kk) of step u of chunk ch (clamped into the year)
    auto kent = [&](const Item &it, uint32_t ch, uint32_t u) {
        const uint32_t c = ch < it.nch ? ch : it.nch - 1;
        return it.kl[(c * kMmaU + u) * 4 + kk];
    };
    // (32-bit byte offsets from uniform bases: the loads take the scalar-base
    // form, with no 64-bit address arithmetic per lane)
    auto dsc = [&](const Item &it, uint2 en) {
        const uint32_t k = (en.y >> 21) & 0xffu;
        return *(const uint32_t *)((const char *)it.dt + ((k << (it.sh + 2)) + it.lc4));
    };
    // C[(k, m)][l]: the slot of Q_kl[m], or the Q row's zero slot (ldQ > ncoef;
    // absent transitions' descriptors name it with nX = 0)
    auto cval = [&](uint2 en, uint32_t d) {
        const uint32_t m = (en.y >> 16) & 31u;
        return *(const double *)((const char *)q + ((m <= ((d >> kOffBits) & 31u) ? (d & kOffMask) + m : zslot) << 3));
    };
    // rings by chunk position j = ch - cb (mod 4 / mod 2): K entries of ch ..
    // ch + 3, descriptors of ch + 1 and ch + 2, C values of ch and ch + 1
    uint2 ee[4][kMmaU];
    uint32_t dd[2][kMmaU];
    double bb[2][kMmaU];
    // an item's first chunks, in two parts: the K entries and descriptors
    // (prime_a), the first C gathers once the descriptors are in (prime_b)
    auto prime_a = [&](const Item &it) {
#pragma unroll
        for (uint32_t u = 0; u < kMmaU; ++u) {
            ee[0][u] = kent(it, it.cb, u);
            ee[1][u] = kent(it, it.cb + 1, u);
            ee[2][u] = kent(it, it.cb + 2, u);
        }
#pragma unroll
        for (uint32_t u = 0; u < kMmaU; ++u) {
            dd[0][u] = dsc(it, ee[0][u]);
            dd[1][u] = dsc(it, ee[1][u]);
        }
    };
    auto prime_b = [&]() {
#pragma unroll
        for (uint32_t u = 0; u < kMmaU; ++u) bb[0][u] = cval(ee[0][u], dd[0][u]);
    };
    Item cur = plan(tmax > 1 ? 1u : 0u);
    if (tmax > 1 && cur.active) {
        prime_a(cur);
        prime_b();
    }
    for (uint32_t t = 1; t < tmax; ++t) {
        mdp_d4 acc[RT];
#pragma unroll
        for (uint32_t h = 0; h < RT; ++h) acc[h] = mdp_d4{0.0, 0.0, 0.0, 0.0};
        // one chunk at ring position j: the K entries of ch + 3, the
        // descriptors of ch + 2, the C values of ch + 1, then ch's products (W
        // formed unconditionally: padded entries name row 0 and meet C = 0)
        auto chunk = [&](uint32_t ch, auto jc) {
            constexpr uint32_t j = decltype(jc)::value;
#pragma unroll
            for (uint32_t u = 0; u < kMmaU; ++u) ee[(j + 3) & 3][u] = kent(cur, ch + 3, u);
#pragma unroll
            for (uint32_t u = 0; u < kMmaU; ++u) dd[j & 1][u] = dsc(cur, ee[(j + 2) & 3][u]);
#pragma unroll
            for (uint32_t u = 0; u < kMmaU; ++u) bb[(j + 1) & 1][u] = cval(ee[(j + 1) & 3][u], dd[(j + 1) & 1][u]);
#pragma unroll
            for (uint32_t u = 0; u < kMmaU; ++u) {
                const uint2 en = ee[j][u];
#pragma unroll
                for (uint32_t h = 0; h < RT; ++h) {
                    const uint32_t pb = (h * 16 + col) * 8u;
                    const double wt = *(const double *)((const char *)xp + (en.x >> 16) + pb) *
                                      *(const double *)((const char *)yp + (en.y & 0xffffu) + pb);
                    const double av = *(const double *)((const char *)Va + (en.x & 0xffffu) + pb) * wt;
                    acc[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(bb[j & 1][u], av, acc[h], 0, 0, 0);
                }
            }
        };
        if (cur.active)
        {
            // whole rounds of four chunks with no branch between them (a
            // branch join made the compiler wait for every load in flight at
            // each chunk), then the last one to three
            uint32_t ch = cur.cb;
            for (; ch + 4 <= cur.ce; ch += 4) {
                chunk(ch, std::integral_constant<uint32_t, 0>{});
                chunk(ch + 1, std::integral_constant<uint32_t, 1>{});
                chunk(ch + 2, std::integral_constant<uint32_t, 2>{});
                chunk(ch + 3, std::integral_constant<uint32_t, 3>{});
            }
            if (ch < cur.ce) chunk(ch, std::integral_constant<uint32_t, 0>{});
            if (ch + 1 < cur.ce) chunk(ch + 1, std::integral_constant<uint32_t, 1>{});
            if (ch + 2 < cur.ce) chunk(ch + 2, std::integral_constant<uint32_t, 2>{});
        }
        // next year's first chunks in flight across this year's barriers
        // (its K entries were staged a year ago): descriptors now, C values
        // after the partial sums
        const Item nxt = plan(t + 1 < tmax ? t + 1 : t);
        const bool pnext = t + 1 < tmax && nxt.active;
        if (pnext) prime_a(nxt);
        // the lane's accumulators: states item * 16 + kk + 4 r of point
        // h * 16 + col; slice 1 stores them in place, slice j >= 2 past row
        // npcp ((S - 2) x ncol x 16 PTS doubles at most, within the buffer)
        double *dst = Vb + (size_t)(cur.item * 16 + kk) * PTS + col;
        auto part = [&](uint32_t j) {
            return Vb + (size_t)cur.npcp * PTS + (size_t)((j - 2) * cur.nit + cur.item) * (RT * 256) + lane;
        };
        if (cur.active && cur.ks == 1)
#pragma unroll
            for (uint32_t h = 0; h < RT; ++h)
#pragma unroll
                for (uint32_t r = 0; r < 4; ++r) dst[(size_t)(4 * r) * PTS + h * 16] = acc[h][r];
        if (cur.active && cur.ks >= 2) {
            double *pk = part(cur.ks);
#pragma unroll
            for (uint32_t h = 0; h < RT; ++h)
#pragma unroll
                for (uint32_t r = 0; r < 4; ++r) pk[(h * 4 + r) * 64] = acc[h][r];
        }
        if (cur.S > 1) __syncthreads();
        if (cur.active && cur.ks == 0) {
            if (cur.S > 1)
#pragma unroll
                for (uint32_t h = 0; h < RT; ++h)
#pragma unroll
                    for (uint32_t r = 0; r < 4; ++r) acc[h][r] = acc[h][r] + dst[(size_t)(4 * r) * PTS + h * 16];
            for (uint32_t j = 2; j < cur.S; ++j) {
                const double *pj = part(j);
#pragma unroll
                for (uint32_t h = 0; h < RT; ++h)
#pragma unroll
                    for (uint32_t r = 0; r < 4; ++r) acc[h][r] = acc[h][r] + pj[(h * 4 + r) * 64];
            }
            // (padded states l >= npc hold 0: their C values are the zero slot)
#pragma unroll
            for (uint32_t h = 0; h < RT; ++h)
#pragma unroll
                for (uint32_t r = 0; r < 4; ++r) dst[(size_t)(4 * r) * PTS + h * 16] = acc[h][r];
        }
        if (pnext) prime_b();
        __syncthreads();
        double *tv = Va;
        Va = Vb;
        Vb = tv;
        cur = nxt;
    }
    if (threadIdx.x < PTS) {
        const uint32_t ie = p0 + threadIdx.x, npl = np[tmax - 1];
        double L = 0.0;
        for (uint32_t l = 0; l < npl; ++l) L += Va[l * PTS + threadIdx.x] * prior0;
        if (ie < ne) out[(size_t)ie * ld_out + (size_t)ic * out_cs] = log(L);
    }
}

// k_fwd_mmt<RT, ROWS, DB> (round 6): the per-year GEMM of k_fwd_mma, for
// years of up to 1 024 states, with three changes.
//  * K lists per (year, column tile): the entry (k, m) only for m <= the
//    largest nX over the tile's 16 new states (k_fwd_mma ran m up to |A_k|
//    for every tile and multiplied the rest through zero slots), and the
//    gathers' Q-row offsets per (entry, new state) from a host table, so no
//    descriptor lookup sits between a K entry and its gather.
//  * Years of more than 128 states (ROWS 256 / 512 / 1 024, 32 / 32 / 16
//    points a block): ONE state buffer in LDS (DB = false, 64 / 128 / 128
//    KiB): a wave keeps its tiles' new states in registers until every wave
//    has read the year's old ones (a barrier), then stores them in place.  A
//    wave owns up to ROWS / 256 tiles a year (17-64 tiles over 16 waves,
//    longest lists first).  Years of up to 128 states keep k_fwd_mma's two
//    buffers (DB = true, 64 points a block, one barrier a year).
//  * Years of at most 16 tiles give every tile a wave and the spare waves to
//    the tiles with the longest lists (a tile's list split into slices of at
//    least two chunks); slice 1 parks its partial products in the tile's own
//    destination rows (two buffers) or past the year's tiles (one buffer),
//    later slices past the year's tiles, and slice 0 adds them in slice
//    order after a barrier (deterministic).
// Workgroups are dealt XCD-aware (the point blocks of one column on one XCD,
// so the column's Q row is gathered from that XCD's L2).  The products sum
// in another order than k_fwd_wide's (positive terms: ~1e-15 relative).
// K steps (of 4 entries) per pipeline chunk: 2, or 1 with 4 point tiles
// (their 4 W operands a step leave no registers for a second step in flight)
constexpr uint32_t mmt_u(uint32_t rt) { return rt == 4 ? 1u : 2u; }
constexpr uint32_t kMmtMaxTiles = 64;   // column tiles a year (1 024 states)
constexpr uint32_t mmt_pts(uint32_t rt) { return 16u * rt; }
// power-table row stride (doubles): rows r and r + 1 on different LDS bank halves
constexpr uint32_t mmt_ps(uint32_t rt) { return rt % 2 ? 16u * rt : 16u * rt + 16u; }
// the instantiations (RT point tiles of 16, ROWS state rows, two buffers or
// one): <4, 128, true> years of up to 128 states, <2, 256, false> 256,
// <2, 512, false> 512, <1, 1 024, false> 1 024 (mmt_shape)
template <int RT, int ROWS, bool DB>
__global__ __launch_bounds__(kMmaThreads) void k_fwd_mmt(
    const double *__restrict__ Q, uint32_t ldQ, const uint32_t *__restrict__ np, const uint2 *__restrict__ kt,
    const uint32_t *__restrict__ cidx, const uint2 *__restrict__ ktile, const uint2 *__restrict__ wplan, uint32_t tmax,
    double prior0, const double *__restrict__ evals, uint32_t ne, uint32_t maxA, double *__restrict__ out,
    uint32_t ld_out, uint32_t out_cs)
{
    constexpr uint32_t PTS = mmt_pts(RT), PS = mmt_ps(RT), TMAX = ROWS > 256 ? ROWS / 256 : 1, U = mmt_u(RT);
    static_assert(TMAX * RT <= 4 && (ROWS <= 256 || TMAX * 256 == ROWS), "tiles per wave");
    extern __shared__ __attribute__((aligned(16))) double mlds[];
    double *Va = mlds, *Vb = DB ? mlds + (size_t)ROWS * PTS : mlds;  // [state][point]: read / written
    double *xp = mlds + (DB ? 2 : 1) * (size_t)ROWS * PTS, *yp = xp + (size_t)(maxA + 1) * PS;  // [r][point]
    const uint32_t lane = threadIdx.x & 63u, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // XCD-aware: workgroups are dealt round-robin over the 8 XCDs; XCD x
    // takes a contiguous range of logical blocks, i.e. whole columns
    const uint32_t npb = (ne + PTS - 1) / PTS, full = gridDim.x & ~7u, b = blockIdx.x;
    const uint32_t lb = b < full ? (b & 7u) * (full >> 3) + (b >> 3) : b;
    const uint32_t p0 = (lb % npb) * PTS, ic = lb / npb;
    if (threadIdx.x < PTS) {
        const uint32_t ie = p0 + threadIdx.x;
        const double e = ie < ne ? evals[ie] : 0.0;
        const double x = e > 1.0 ? 1.0 : e, y = 1.0 - x;
        double a = 1.0, c = 1.0;
        for (uint32_t r = 0; r <= maxA; ++r) {
            xp[r * PS + threadIdx.x] = a;
            yp[r * PS + threadIdx.x] = c;
            a *= x;
            c *= y;
        }
    }
    const uint32_t np0 = np[0];
    for (uint32_t i = threadIdx.x; i < ROWS * PTS; i += kMmaThreads) Va[i] = i / PTS < np0 ? 1.0 : 0.0;
    __syncthreads();
    const double *q = Q + (size_t)ic * ldQ;
    const uint32_t kk = lane >> 4, col = lane & 15u;
    struct Item {
        uint32_t tile, ks, S, pbase, cb, ce, nch, npcp;
        bool active, split;
        const uint2 *kl;
        const uint32_t *cl;
    };
    // item i of this wave in year t (host table mmt_wplan: no divisions here)
    auto plan = [&](uint32_t t, uint32_t i) {
        Item it;
        it.npcp = (np[t] + 15) / 16 * 16;
        const uint2 wp = wplan[(t * 16 + wv) * TMAX + i];
        it.cb = wp.x & 0xffffu;
        it.ce = wp.x >> 16;
        it.tile = wp.y & 0xffu;
        it.ks = (wp.y >> 8) & 15u;      // slice of the tile's K list
        it.S = (wp.y >> 12) & 31u;      // the tile's slices
        it.pbase = (wp.y >> 17) & 31u;  // its partial blocks (slices 1 .. S - 1) from here
        it.split = (wp.y >> 22) & 1u;   // some tile of the year is sliced (uniform)
        it.active = (wp.y >> 24) != 0u;
        const uint2 kt2 = ktile[t * kMmtMaxTiles + it.tile];
        const uint32_t k0 = __builtin_amdgcn_readfirstlane(kt2.x);
        it.kl = kt + k0;
        it.cl = cidx + (size_t)k0 * 16;
        it.nch = kt2.y;
        return it;
    };
    // K entry (uint2, one per 16 lanes): x = V row byte offset (18 bits) |
    // y^m row offset << 18, y = x^(|A|-m) row offset (16 bits) | m << 16 | k
    // << 21; and per lane the byte offset in the Q row of C[(k, m)][l] --
    // Q_kl[m], or the zero slot where m > nX or l is a padded state (host
    // table, so no descriptor lookup is on the gather's path)
    auto kent = [&](const Item &it, uint32_t ch, uint32_t u) {
        const uint32_t c = ch < it.nch ? ch : it.nch - 1;
        return it.kl[(c * U + u) * 4 + kk];
    };
    auto coff = [&](const Item &it, uint32_t ch, uint32_t u) {
        const uint32_t c = ch < it.nch ? ch : it.nch - 1;
        return it.cl[(c * U + u) * 64 + lane];
    };
    auto cval = [&](uint32_t o) { return *(const double *)((const char *)q + o); };
    // rings by chunk position j = ch - cb: K entries of ch .. ch + 3 (mod
    // 4), C offsets of ch + 1 and ch + 2 (mod 2; ch's were consumed by its
    // gathers), C values of ch and ch + 1 (mod 2)
    uint2 ee[4][U];
    uint32_t dd[2][U];
    double bb[2][U];
    auto prime_a = [&](const Item &it) {
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            ee[0][u] = kent(it, it.cb, u);
            ee[1][u] = kent(it, it.cb + 1, u);
            ee[2][u] = kent(it, it.cb + 2, u);
            dd[0][u] = coff(it, it.cb, u);
            dd[1][u] = coff(it, it.cb + 1, u);
        }
    };
    auto prime_b = [&]() {
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) bb[0][u] = cval(dd[0][u]);
    };
    Item cur = plan(tmax > 1 ? 1u : 0u, 0);
    if (tmax > 1 && cur.active) {
        prime_a(cur);
        prime_b();
    }
    for (uint32_t t = 1; t < tmax; ++t) {
        mdp_d4 acc[TMAX][RT];
        const Item first = cur;
#pragma unroll
        for (uint32_t i = 0; i < TMAX; ++i) {
#pragma unroll
            for (uint32_t h = 0; h < RT; ++h) acc[i][h] = mdp_d4{0.0, 0.0, 0.0, 0.0};
            if (i > 0) {
                cur = plan(t, i);
                if (!cur.active) break;  // a wave's items are its first ones
                prime_a(cur);
                prime_b();
            }
            if (!cur.active) break;
            mdp_d4(&ac)[RT] = acc[i];  // (i is a constant once unrolled)
            // one chunk at ring position j: the K entries of ch + 3, the C
            // values of ch + 1 (their offsets loaded a chunk ago), the C
            // offsets of ch + 2, then ch's products
            auto chunk = [&](uint32_t ch, auto jc) {
                constexpr uint32_t j = decltype(jc)::value;
#pragma unroll
                for (uint32_t u = 0; u < U; ++u) ee[(j + 3) & 3][u] = kent(cur, ch + 3, u);
#pragma unroll
                for (uint32_t u = 0; u < U; ++u) bb[(j + 1) & 1][u] = cval(dd[(j + 1) & 1][u]);
#pragma unroll
                for (uint32_t u = 0; u < U; ++u) dd[j & 1][u] = coff(cur, ch + 2, u);
#pragma unroll
                for (uint32_t u = 0; u < U; ++u) {
                    const uint2 en = ee[j][u];
#pragma unroll
                    for (uint32_t h = 0; h < RT; ++h) {
                        const uint32_t pb = (h * 16 + col) * 8u;
                        const double wt = *(const double *)((const char *)xp + (en.y & 0xffffu) + pb) *
                                          *(const double *)((const char *)yp + (en.x >> 18) + pb);
                        const double av = *(const double *)((const char *)Va + (en.x & 0x3ffffu) + pb) * wt;
                        ac[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(bb[j & 1][u], av, ac[h], 0, 0, 0);
                    }
                }
            };
            uint32_t ch = cur.cb;
            for (; ch + 4 <= cur.ce; ch += 4) {
                chunk(ch, std::integral_constant<uint32_t, 0>{});
                chunk(ch + 1, std::integral_constant<uint32_t, 1>{});
                chunk(ch + 2, std::integral_constant<uint32_t, 2>{});
                chunk(ch + 3, std::integral_constant<uint32_t, 3>{});
            }
            if (ch < cur.ce) chunk(ch, std::integral_constant<uint32_t, 0>{});
            if (ch + 1 < cur.ce) chunk(ch + 1, std::integral_constant<uint32_t, 1>{});
            if (ch + 2 < cur.ce) chunk(ch + 2, std::integral_constant<uint32_t, 2>{});
        }
        // next year's first item: K entries and descriptors in flight across
        // this year's barriers, its first C values after them
        const Item nxt = plan(t + 1 < tmax ? t + 1 : t, 0);
        const bool pnext = t + 1 < tmax && nxt.active;
        if (pnext) prime_a(nxt);
        if constexpr (!DB) __syncthreads();  // one buffer: every wave has read the year's old states
        // the lane's accumulators: states tile * 16 + kk + 4 r of point
        // h * 16 + col.  A sliced tile's slices ks >= 1 park theirs: slice 1
        // of two buffers in the tile's destination rows, the rest past row
        // npcp in partial block pbase + ks - (DB ? 2 : 1) of the year (the
        // host keeps them within ROWS rows)
        auto dst_of = [&](uint32_t tile) { return Vb + (size_t)(tile * 16 + kk) * PTS + col; };
        auto park = [&](uint32_t ks) {
            return Vb + (size_t)(first.npcp + (first.pbase + ks - (DB ? 2u : 1u)) * 16) * PTS + lane;
        };
        if (first.split) {
            if (first.active && first.ks >= 1) {
                if (DB && first.ks == 1) {
                    double *dst = dst_of(first.tile);
#pragma unroll
                    for (uint32_t h = 0; h < RT; ++h)
#pragma unroll
                        for (uint32_t r = 0; r < 4; ++r) dst[(size_t)(4 * r) * PTS + h * 16] = acc[0][h][r];
                } else {
                    double *pk = park(first.ks);
#pragma unroll
                    for (uint32_t h = 0; h < RT; ++h)
#pragma unroll
                        for (uint32_t r = 0; r < 4; ++r) pk[(h * 4 + r) * 64] = acc[0][h][r];
                }
            }
            __syncthreads();
            if (first.active && first.ks == 0)
                for (uint32_t j = 1; j < first.S; ++j) {
                    if (DB && j == 1) {
                        const double *dst = dst_of(first.tile);
#pragma unroll
                        for (uint32_t h = 0; h < RT; ++h)
#pragma unroll
                            for (uint32_t r = 0; r < 4; ++r)
                                acc[0][h][r] = acc[0][h][r] + dst[(size_t)(4 * r) * PTS + h * 16];
                    } else {
                        const double *pj = park(j);
#pragma unroll
                        for (uint32_t h = 0; h < RT; ++h)
#pragma unroll
                            for (uint32_t r = 0; r < 4; ++r) acc[0][h][r] = acc[0][h][r] + pj[(h * 4 + r) * 64];
                    }
                }
            // (the final stores below go to rows < npcp, never to a parked
            // block, and a tile's slice-1 rows are read only by its slice 0)
        }
        // (padded states l >= npc hold 0: their C values are the zero slot)
#pragma unroll
        for (uint32_t i = 0; i < TMAX; ++i) {
            const Item it = i == 0 ? first : plan(t, i);
            if (!it.active || it.ks != 0) break;
            double *dst = dst_of(it.tile);
#pragma unroll
            for (uint32_t h = 0; h < RT; ++h)
#pragma unroll
                for (uint32_t r = 0; r < 4; ++r) dst[(size_t)(4 * r) * PTS + h * 16] = acc[i][h][r];
        }
        if (pnext) prime_b();
        __syncthreads();
        if constexpr (DB) {
            double *tv = Va;
            Va = Vb;
            Vb = tv;
        }
        cur = nxt;
    }
    if (threadIdx.x < PTS) {
        const uint32_t ie = p0 + threadIdx.x, npl = np[tmax - 1];
        double L = 0.0;
        for (uint32_t l = 0; l < npl; ++l) L += Va[l * PTS + threadIdx.x] * prior0;
        if (ie < ne) out[(size_t)ie * ld_out + (size_t)ic * out_cs] = log(L);
    }
}

// k_fwd_hs<RT, NB, NW> (round 6): the wide forward through the hidden
// states.  The reference's own factorisation (main_MIDASPOM.c:18-50, :363,
// :371-384): P = Pe Pc over the hidden states j, so year t is
//     U[p][j] = y^|j| sum_{k: A_k >= j} v[p][k] x^(|A_k| - |j|)    (v Pe)
//     n[p][l] = sum_{j <= B_l} Pc[j][B_l] U[p][j]                  (U Pc)
// instead of one (nX+1)-term polynomial per transition (k, l): for a year of
// 2^f completions of f unvisited patches that is ~3^f (j, l) terms per
// point, not ~2^f 2^f (|A|+1) -- 10-25x fewer for years of 256-1 024 states.
// An NW-wave block's 16 RT points keep one vector over the whole 2^NB cube
// of hidden states in LDS, V[j][p] (NB = max(8, nvar) <= 10; 64 or 128 KiB),
// plus a y^k table:
//  * v Pe: Pe is a tensor product over the patches (per patch: occupied ->
//    extinct w.p. x, survives w.p. y), applied in place by passes of up to
//    kHsRadix patches of W = the bits occupied in some state of year t - 1:
//    a thread loads a coset's positions, runs the butterflies V[j] +=
//    x V[j | b] in registers and writes back, y^|j| applied in the year's
//    last pass.  The host's pass tables (build_hs_plan) name per coset the
//    positions to read and to write -- only those whose value still reaches
//    a hidden state the year's products read -- and give a wave's cosets the
//    same masks, so uniform branches skip the rest;
//  * U Pc: the per-year GEMM on the matrix cores as k_fwd_mmt's, with K = the
//    hidden states j a column tile of new states reaches, the W operand
//    U[j][p] read straight from the cube, and the C operand Pc[j][B_l]
//    gathered from the column's item factors (k_witems' Pg rows, ld =
//    nitems + 1: a zero slot at nitems for j not <= B_l) through a host
//    table of offsets;
//  * the year's new states are stored at their own cube positions B_l (after
//    a barrier: U is dead by then), ready for the next year's passes.
// Tiles are dealt to waves as k_fwd_mmt's (longest lists first past NW
// tiles; smaller years give the spare waves slices of the longest lists,
// parked in 16-row cube blocks that hold none of the year's states).  Q3
// semantics: ones at year 0's states; L = prior0 x the sum over the last
// year's states.  Sums reordered against the reference's (positive terms
// for e in [0, 1]: ~1e-15 relative).
constexpr uint32_t kHsRadix = 4;  // k_fwd_hs: patches per v Pe pass (at most; the plan's default)
constexpr uint32_t kHsPre = 4;    // k_fwd_hs: v Pe passes a year whose descriptors are loaded up front
// diag build, MDP_HS_PROBE bit 2: workgroup 0's wave 0 stamps the shader
// clock at each phase of each year into out[] (results not stored)
#ifdef MDP_DIAG_BUILD
#define MDP_HS_STAMP(k)                                                                                      \
    do {                                                                                                     \
        if ((probe & 4u) && blockIdx.x == 0 && threadIdx.x == 0) out[(size_t)t * 8 + (k)] = (double)clock64(); \
    } while (0)
#else
#define MDP_HS_STAMP(k) do { } while (0)
#endif
template <int RT, int NB, int NW>
__global__ __launch_bounds__(NW * 64, 4) void k_fwd_hs(  // (4 waves a SIMD: two 8-wave blocks a CU)
    const double *__restrict__ Pg, uint32_t ldp, uint32_t c0, const uint32_t *__restrict__ np,
    const uint32_t *__restrict__ kt, const uint32_t *__restrict__ cidx, const uint4 *__restrict__ wplan,
    const uint4 *__restrict__ pass, const uint32_t *__restrict__ pbase, const uint2 *__restrict__ ppos, const uint32_t *__restrict__ dpos, const uint32_t *__restrict__ dbase,
    const uint2 *__restrict__ dpk, const uint32_t *__restrict__ pk, uint32_t tmax, double prior0, const double *__restrict__ evals, uint32_t ne,
    double *__restrict__ out, uint32_t ld_out, uint32_t out_cs, uint32_t probe)
{
    constexpr uint32_t PTS = mmt_pts(RT), NC = 1u << NB, NTH = NW * 64, TMAX = NC / 16 > NW ? NC / 16 / NW : 1,
                       U = mmt_u(RT);
    static_assert(TMAX * RT <= 4 && NC * PTS <= 16384 && NTH % PTS == 0, "cube and tiles");
    extern __shared__ __attribute__((aligned(16))) double mlds[];
    double *V = mlds;  // [j][point]
    const uint32_t lane = threadIdx.x & 63u, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // XCD-aware: XCD x takes a contiguous range of logical blocks (whole columns)
    const uint32_t npb = (ne + PTS - 1) / PTS, full = gridDim.x & ~7u, b = blockIdx.x;
    const uint32_t lb = b < full ? (b & 7u) * (full >> 3) + (b >> 3) : b;
    const uint32_t p0 = (lb % npb) * PTS, cl = lb / npb, ic = c0 + cl;
    // this thread's point in the pass loops (NTH is a multiple of PTS)
    const uint32_t pp = threadIdx.x % PTS;
    double xq, yq;
    {
        const uint32_t ie = p0 + pp;
        const double e = ie < ne ? evals[ie] : 0.0;
        xq = e > 1.0 ? 1.0 : e;
        yq = 1.0 - xq;
    }
    // the cube starts at zero (a position no year has written holds a finite
    // value whenever it is read: padded K entries meet it with C = 0), then
    // ones at year 0's states (Q3)
    for (uint32_t i = threadIdx.x; i < NC * PTS; i += NTH) V[i] = 0.0;
    __syncthreads();
    {
        const uint32_t n0 = (np[0] + 15) / 16 * 16, d0 = dbase[0];
        for (uint32_t i = threadIdx.x; i < n0 * PTS; i += NTH) {
            const uint32_t pos = dpos[d0 + i / PTS];
            if (pos != ~0u) V[pos * PTS + i % PTS] = 1.0;
        }
    }
    __syncthreads();
    const double *q = Pg + (size_t)cl * ldp;
    const uint32_t kk = lane >> 4, col = lane & 15u;
    struct Item {
        uint32_t tile, ks, S, pbase, cb, ce, nch;
        bool active, split;
        const uint32_t *kl, *cl;
    };
    // item i of this wave in year t (wplan: chunk range, tile | slice |
    // slices | park base | split | valid, the tile's K-list start and
    // chunks: one scalar load, no dependent one)
    auto plan = [&](uint32_t t, uint32_t i) {
        Item it;
        const uint4 wp = wplan[(t * NW + wv) * TMAX + i];
        it.cb = wp.x & 0xffffu;
        it.ce = wp.x >> 16;
        it.tile = wp.y & 0xffu;
        it.ks = (wp.y >> 8) & 15u;
        it.S = (wp.y >> 12) & 31u;
        it.pbase = (wp.y >> 17) & 31u;
        it.split = (wp.y >> 22) & 1u;
        it.active = (wp.y >> 24) != 0u;
        const uint32_t k0 = __builtin_amdgcn_readfirstlane(wp.z);
        it.kl = kt + k0;
        it.cl = cidx + (size_t)k0 * 16;
        it.nch = wp.w;
        return it;
    };
    // K entry (one per 16 lanes): the LDS byte offset of U's row j; per lane
    // the byte offset of Pc[j][B_l] in the column's Pg row (or its zero slot)
    auto kent = [&](const Item &it, uint32_t ch, uint32_t u) {
        const uint32_t c = ch < it.nch ? ch : it.nch - 1;
        return it.kl[(c * U + u) * 4 + kk];
    };
    auto coff = [&](const Item &it, uint32_t ch, uint32_t u) {
        const uint32_t c = ch < it.nch ? ch : it.nch - 1;
        return it.cl[(c * U + u) * 64 + lane];
    };
    auto cval = [&](uint32_t o) { return *(const double *)((const char *)q + o); };
    uint32_t ee[4][U];
    uint32_t dd[2][U];
    double bb[2][U];
    auto prime = [&](const Item &it) {
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            ee[0][u] = kent(it, it.cb, u);
            ee[1][u] = kent(it, it.cb + 1, u);
            ee[2][u] = kent(it, it.cb + 2, u);
            dd[0][u] = coff(it, it.cb, u);
            dd[1][u] = coff(it, it.cb + 1, u);
        }
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) bb[0][u] = cval(dd[0][u]);
    };
    // y^k of the thread's point (the v Pe passes' last scaling)
    double *ypw = mlds + (size_t)NC * PTS;  // [k][point], k <= NB
    if (threadIdx.x < PTS) {
        double a = 1.0;
        for (uint32_t k = 0; k <= (uint32_t)NB; ++k, a *= yq) ypw[k * PTS + threadIdx.x] = a;
    }
    __syncthreads();
    // one coset of a v Pe pass (R patches, bit masks mb): read the positions
    // of mask inm (the rest count as 0), the R butterflies V[j] += x V[j | b]
    // in registers, write the positions of mask outm (those some later pass
    // or the year's products read) -- in the year's last pass times y^|j|
    // (a wave's cosets share their masks, build_hs_plan: uniform branches
    // skip the positions no lane of the wave reads or writes)
    auto coset = [&](auto rc, uint2 ce, const uint32_t (&mb)[kHsRadix], bool last) {
        constexpr uint32_t R = decltype(rc)::value, NQ = 1u << R;
        const uint32_t my = __builtin_amdgcn_readfirstlane(ce.y);
        const uint32_t g = ce.x, inm = my & 0xffffu, outm = my >> 16;
        auto pos = [&](uint32_t qq) {
            uint32_t o = g;
#pragma unroll
            for (uint32_t k = 0; k < R; ++k) o |= (qq >> k) & 1u ? mb[k] : 0u;
            return o;
        };
        double v[NQ];
#pragma unroll
        for (uint32_t qq = 0; qq < NQ; ++qq) {
            if ((inm >> qq) & 1u)
                v[qq] = V[(size_t)pos(qq) * PTS + pp];
            else
                v[qq] = 0.0;
        }
#pragma unroll
        for (uint32_t k = 0; k < R; ++k)
#pragma unroll
            for (uint32_t qq = 0; qq < NQ; ++qq)
                if (qq & (1u << k)) v[qq ^ (1u << k)] = fma(xq, v[qq], v[qq ^ (1u << k)]);
        if (last) {
            double sc[R + 1];
            sc[0] = ypw[__builtin_popcount(g) * PTS + pp];
#pragma unroll
            for (uint32_t k = 1; k <= R; ++k) sc[k] = sc[k - 1] * yq;
#pragma unroll
            for (uint32_t qq = 0; qq < NQ; ++qq) v[qq] *= sc[__builtin_popcount(qq)];
        }
#pragma unroll
        for (uint32_t qq = 0; qq < NQ; ++qq)
            if ((outm >> qq) & 1u) V[(size_t)pos(qq) * PTS + pp] = v[qq];
    };
    // v Pe pass tables of a year: the pass range, the first kHsPre passes'
    // descriptors and this thread's first coset of each -- loaded a year
    // ahead (during the previous year's products), so no year waits on them
    const uint32_t i0 = threadIdx.x / PTS;
    uint32_t pb0 = 0, pb1 = 0;
    uint4 pdp[kHsPre];
    uint2 cep[kHsPre];
    auto load_passes = [&](uint32_t ty) {
        pb0 = pbase[ty];
        pb1 = (probe & 1u) ? pb0 : pbase[ty + 1];
#pragma unroll
        for (uint32_t k = 0; k < kHsPre; ++k)
            if (pb0 + k < pb1) {
                pdp[k] = pass[pb0 + k];
                cep[k] = i0 < pdp[k].z ? ppos[pdp[k].w + i0] : make_uint2(0u, 0u);
            }
    };
    if (tmax > 1) load_passes(1);
    for (uint32_t t = 1; t < tmax; ++t) {
        // the year's first work item: its K entries, C offsets and first C
        // values do not depend on the cube, so their loads are in flight
        // through the v Pe passes; so are the positions its new states are
        // stored at (dpk: 4 x 16 bits per lane and tile, 0xffff: padding)
        mdp_d4 acc[TMAX][RT];
        Item cur = plan(t, 0);
        const Item first = cur;
        if (cur.active && !(probe & 2u)) prime(cur);
        const uint32_t db = dbase[t];
        uint2 dk[TMAX];
#pragma unroll
        for (uint32_t i = 0; i < TMAX; ++i) {
            const uint4 w2 = wplan[(t * NW + wv) * TMAX + i];
            dk[i] = (w2.y >> 24) ? dpk[(db / 16 + (w2.y & 0xffu)) * 4 + kk] : make_uint2(~0u, ~0u);
        }
        // v Pe: U[j] = y^|j| sum_{A >= j} v[A] x^(|A| - |j|), the patches of
        // W up to kHsRadix at a time (pass table: the r patches' bit
        // positions, r, cosets, coset-list base)
        MDP_HS_STAMP(0);
        for (uint32_t ps = pb0; ps < pb1; ++ps) {
            const uint32_t k0 = ps - pb0;
            if (ps == pb0) MDP_HS_STAMP(1);
            uint4 pd;
            if (k0 < kHsPre) {
                pd = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
                for (uint32_t k = 0; k < kHsPre; ++k)
                    if (k == k0) pd = pdp[k];
            } else {
                pd = pass[ps];
            }
            const uint32_t r = pd.y, ncos = pd.z, base = pd.w;
            const bool last = ps + 1 == pb1;
            uint32_t mb[kHsRadix];
#pragma unroll
            for (uint32_t k = 0; k < kHsRadix; ++k) mb[k] = k < r ? 1u << ((pd.x >> (5 * k)) & 31u) : 0u;
            for (uint32_t i = i0; i < ncos; i += NTH / PTS) {
                uint2 ce;
                if (i == i0 && k0 < kHsPre) {
                    ce = make_uint2(0u, 0u);
#pragma unroll
                    for (uint32_t k = 0; k < kHsPre; ++k)
                        if (k == k0) ce = cep[k];
                } else {
                    ce = ppos[base + i];
                }
                if (r == 4) coset(std::integral_constant<uint32_t, 4>{}, ce, mb, last);
                else if (r == 3) coset(std::integral_constant<uint32_t, 3>{}, ce, mb, last);
                else if (r == 2) coset(std::integral_constant<uint32_t, 2>{}, ce, mb, last);
                else coset(std::integral_constant<uint32_t, 1>{}, ce, mb, last);
            }
            __syncthreads();
        }
        MDP_HS_STAMP(2);
        // U Pc on the matrix cores
#pragma unroll
        for (uint32_t i = 0; i < TMAX; ++i) {
#pragma unroll
            for (uint32_t h = 0; h < RT; ++h) acc[i][h] = mdp_d4{0.0, 0.0, 0.0, 0.0};
            if (i > 0) cur = plan(t, i);
            if (!cur.active || (probe & 2u)) break;  // a wave's items are its first ones
            if (i > 0) prime(cur);
            mdp_d4(&ac)[RT] = acc[i];  // (i is a constant once unrolled)
            auto chunk = [&](uint32_t ch, auto jc) {
                constexpr uint32_t j = decltype(jc)::value;
#pragma unroll
                for (uint32_t u = 0; u < U; ++u) ee[(j + 3) & 3][u] = kent(cur, ch + 3, u);
#pragma unroll
                for (uint32_t u = 0; u < U; ++u) bb[(j + 1) & 1][u] = cval(dd[(j + 1) & 1][u]);
#pragma unroll
                for (uint32_t u = 0; u < U; ++u) dd[j & 1][u] = coff(cur, ch + 2, u);
#pragma unroll
                for (uint32_t u = 0; u < U; ++u) {
                    const uint32_t joff = ee[j][u];
#pragma unroll
                    for (uint32_t h = 0; h < RT; ++h) {
                        const double av = *(const double *)((const char *)V + joff + (h * 16 + col) * 8u);
                        ac[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(bb[j & 1][u], av, ac[h], 0, 0, 0);
                    }
                }
            };
            uint32_t ch = cur.cb;
            for (; ch + 4 <= cur.ce; ch += 4) {
                chunk(ch, std::integral_constant<uint32_t, 0>{});
                chunk(ch + 1, std::integral_constant<uint32_t, 1>{});
                chunk(ch + 2, std::integral_constant<uint32_t, 2>{});
                chunk(ch + 3, std::integral_constant<uint32_t, 3>{});
            }
            if (ch < cur.ce) chunk(ch, std::integral_constant<uint32_t, 0>{});
            if (ch + 1 < cur.ce) chunk(ch + 1, std::integral_constant<uint32_t, 1>{});
            if (ch + 2 < cur.ce) chunk(ch + 2, std::integral_constant<uint32_t, 2>{});
        }
        MDP_HS_STAMP(3);
        if (t + 1 < tmax) load_passes(t + 1);
        __syncthreads();  // every wave has read U
        MDP_HS_STAMP(4);
        // the lane's accumulators: new states tile * 16 + kk + 4 r (tile
        // order) of point h * 16 + col
        auto store = [&](uint2 d2, const mdp_d4 (&a)[RT]) {
#pragma unroll
            for (uint32_t r = 0; r < 4; ++r) {
                const uint32_t pos = ((r < 2 ? d2.x : d2.y) >> (16 * (r & 1))) & 0xffffu;
                if (pos == 0xffffu) continue;
                double *dst = V + (size_t)pos * PTS + col;
#pragma unroll
                for (uint32_t h = 0; h < RT; ++h) dst[h * 16] = a[h][r];
            }
        };
        // a sliced tile's slices ks >= 1 park their partials in 16-row
        // blocks of the cube that hold none of the year's states (host table
        // pk: U is dead, and the next year's butterflies write such a
        // position before reading it); slice 0 adds them in slice order
        if (first.split) {
            auto park = [&](uint32_t ks) { return V + (size_t)pk[t * 16 + first.pbase + ks - 1] * PTS + lane; };
            if (first.active && first.ks >= 1) {
                double *pkp = park(first.ks);
#pragma unroll
                for (uint32_t h = 0; h < RT; ++h)
#pragma unroll
                    for (uint32_t r = 0; r < 4; ++r) pkp[(h * 4 + r) * 64] = acc[0][h][r];
            }
            __syncthreads();
            if (first.active && first.ks == 0)
                for (uint32_t j = 1; j < first.S; ++j) {
                    const double *pj = park(j);
#pragma unroll
                    for (uint32_t h = 0; h < RT; ++h)
#pragma unroll
                        for (uint32_t r = 0; r < 4; ++r) acc[0][h][r] = acc[0][h][r] + pj[(h * 4 + r) * 64];
                }
            __syncthreads();  // parked blocks read before any tile's store
        }
#pragma unroll
        for (uint32_t i = 0; i < TMAX; ++i) {
            const Item it = i == 0 ? first : plan(t, i);
            if (!it.active || it.ks != 0) break;
            store(dk[i], acc[i]);
        }
        MDP_HS_STAMP(5);
        __syncthreads();
        MDP_HS_STAMP(6);
    }
    if (threadIdx.x < PTS && !(probe & 4u)) {
        const uint32_t ie = p0 + threadIdx.x, dl = dbase[tmax - 1], npl = (np[tmax - 1] + 15) / 16 * 16;
        double L = 0.0;
        for (uint32_t l = 0; l < npl; ++l) {
            const uint32_t pos = dpos[dl + l];
            if (pos != ~0u) L += V[pos * PTS + threadIdx.x] * prior0;
        }
        if (ie < ne) out[(size_t)ie * ld_out + (size_t)ic * out_cs] = log(L);
    }
}

typedef const __attribute__((address_space(4))) uint32_t cuint;

// Forward recursion with the state vectors in HBM: lane per e value, one c
// per workgroup row (blockIdx.y = c0 + row).  Year t's vector is formed
// kWideLB target states at a time, each source state's probability loaded
// once per block of targets; a transition's coefficients (its group's Q
// entries) and its use descriptor are wave-uniform scalar loads.  The weight
// x^(|A|-m) y^m is xp[|A|-m] yp[m] from per-lane power tables in LDS.  Q3
// semantics (:368-369, :386-392): ones over the year-0 states, L = prior0 sum v.
constexpr uint32_t kWideLB = 4;
__global__ __launch_bounds__(kBlock) void k_fwd_wide(
    const double *__restrict__ Q, uint32_t ldQ, const uint32_t *__restrict__ udesc,
    const uint32_t *__restrict__ np, uint32_t tmax, double prior0, const double *__restrict__ evals, uint32_t ne,
    uint32_t c0, uint32_t maxA, double *__restrict__ V, uint32_t npmax, double *__restrict__ out, uint32_t ld_out,
    uint32_t out_cs)
{
    extern __shared__ double xy[];  // [2][maxA + 1][kBlock]: x^r, y^r per lane
    const uint32_t ie = blockIdx.x * kBlock + threadIdx.x, cl = blockIdx.y, ic = c0 + cl;
    const double e = ie < ne ? evals[ie] : 0.0;
    const double x = e > 1.0 ? 1.0 : e, y = 1.0 - x;
    double *xp = xy + threadIdx.x, *yp = xy + (size_t)(maxA + 1) * kBlock + threadIdx.x;
    {
        double a = 1.0, b = 1.0;
        for (uint32_t r = 0; r <= maxA; ++r) {
            xp[r * kBlock] = a;
            yp[r * kBlock] = b;
            a *= x;
            b *= y;
        }
    }
    cdouble *q = (cdouble *)(Q + (size_t)ic * ldQ);
    cuint *ud = (cuint *)udesc;
    cuint *npc_ = (cuint *)np;
    // V[buf][state][row][lane]: rows of this launch x the padded e extent
    const size_t cs = (size_t)gridDim.y * gridDim.x * kBlock;  // one state's stride
    double *va = V + (size_t)cl * gridDim.x * kBlock + ie;
    double *vb = va + (size_t)npmax * cs;
    const uint32_t np0 = npc_[0];
    for (uint32_t k = 0; k < np0; ++k) va[k * cs] = 1.0;
    uint32_t ubase = 0, npp = np0;
    for (uint32_t t = 1; t < tmax; ++t) {
        const uint32_t npc = npc_[t];
        for (uint32_t l0 = 0; l0 < npc; l0 += kWideLB) {
            double acc[kWideLB];
#pragma unroll
            for (uint32_t i = 0; i < kWideLB; ++i) acc[i] = 0.0;
            for (uint32_t k = 0; k < npp; ++k) {
                const double vk = va[k * cs];
#pragma unroll
                for (uint32_t i = 0; i < kWideLB; ++i) {
                    if (l0 + i >= npc) break;
                    const uint32_t d = ud[ubase + (l0 + i) * npp + k];
                    const uint32_t off = d & kOffMask, nX = (d >> kOffBits) & 31u, nA = d >> 27;
                    double P = 0.0;
                    for (uint32_t m = 0; m <= nX; ++m) P = fma(q[off + m], xp[(nA - m) * kBlock] * yp[m * kBlock], P);
                    acc[i] = fma(vk, P, acc[i]);
                }
            }
#pragma unroll
            for (uint32_t i = 0; i < kWideLB; ++i)
                if (l0 + i < npc) vb[(l0 + i) * cs] = acc[i];
        }
        ubase += npp * npc;
        npp = npc;
        double *tmp = va;
        va = vb;
        vb = tmp;
    }
    double L = 0.0;
    for (uint32_t l = 0; l < npp; ++l) L += va[l * cs] * prior0;
    if (ie < ne) out[(size_t)ie * ld_out + (size_t)ic * out_cs] = log(L);
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

constexpr int kNumEv = 6;  // start/stop per kernel: k_zpv, k_coefs, k_forward
const char *const kKernelNames[3][3] = {{"k_zpv", "k_coefs", "k_forward"},
                                        {"k_zrows", "k_qrows", "k_forward"},
                                        {"k_zrows", "k_witems+k_wq", "k_fwd_wide"}};

struct DevCtx {
    int device = 0;
    hipStream_t stream = nullptr;
    double *S = nullptr;
    uint32_t *var_cols = nullptr, *row_col = nullptr;
    uint32_t *pairA = nullptr, *pairB = nullptr, *pairOff = nullptr;
    uint32_t *udesc = nullptr, *prog = nullptr, *pairPart0 = nullptr, *partP = nullptr, *partK0 = nullptr;
    double *e = nullptr, *c = nullptr;
    size_t cap_e = 0, cap_c = 0;
    uint32_t ne = 0, nc = 0;
    uint32_t ne_sform = 0;  // e rows of this grid on the s-form (x < y), for the work count
    // forward kernels with several points per lane: list positions -> e rows
    // (bit 31: a duplicate that is computed, not stored), grouped by ratio form
    uint32_t *plist = nullptr;
    size_t cap_plist = 0;
    uint32_t nlist = 0, nlist_epl = 0;  // list length (a multiple of nlist_epl, its points per lane)
    bool plist_identity = true;          // the list is 0, 1, ... (nothing uploaded; plist passed as null)
    double *ZPV = nullptr, *R = nullptr, *out = nullptr, *gpart = nullptr;
    size_t cap_zpv = 0, cap_r = 0, cap_out = 0, cap_gpart = 0;
    unsigned long long *stamps[3] = {nullptr, nullptr, nullptr};  // k_zpv, k_coefs, k_forward
    size_t cap_st[3] = {0, 0, 0};
    size_t nst[3] = {0, 0, 0};
    // direct path: k_zrows / k_qrows tables (zs, row-major [row][k], depends
    // on the grid's c range)
    double *zs = nullptr, *sv = nullptr, *Qrow = nullptr, *Zg = nullptr;
    double *zsq = nullptr;  // zs chain-major, [row][k mod 4][k / 4] (k_qrows: a lane's chain contiguous)
    double *zc = nullptr;   // Z-row series coefficients [row][kZTerms]
    size_t cap_zc = 0;
    uint2 *items = nullptr;  // per item {B | row << 24, j | (row >> 8) << 24}
    uint2 *qslot = nullptr;  // k_qrows phase-3 lane table
    uint32_t *qlane = nullptr;  // k_qrows phase-3 Pc slots per lane (nvar <= 8)
    uint32_t *islot = nullptr;  // k_qrows: each item's Pc slot
    uint32_t *itemB = nullptr, *qstart = nullptr, *qitem = nullptr;
    size_t cap_zs = 0, cap_zsq = 0, cap_qrow = 0, cap_zg = 0;
    uint32_t zs_len = 0;    // doubles in zs = zs_kmax * nj
    double *coltab = nullptr;  // fused kernel's column tables (plan offsets, zs last), 1 KiB padded
    size_t cap_coltab = 0;
    uint32_t ct_len = 0;       // doubles
    uint32_t zs_kmax = 0;   // padded length of the longest pruned row
    uint32_t qrows_cb = 1;  // c values per k_qrows workgroup for this grid
    bool qrows_attr_set = false;  // k_qrows' LDS limit raised on this device
    double zs_cmax = -1.0;  // c bound the uploaded zs was pruned for (-1: none yet)
    // problem-specialised forward kernel [variant]: 0 reading, 1 fused, 2
    // reading at kJitKblockTall threads (tall grids, set_grid_dev)
    hipModule_t jit_mod[3] = {nullptr, nullptr, nullptr};
    hipFunction_t jit_fn[3] = {nullptr, nullptr, nullptr};
    // a long series: one forward kernel per chunk of years, the state vector
    // handed over in vscr[state][c][e] (ldv e values per (state, c))
    std::vector<hipModule_t> cmod;
    std::vector<hipFunction_t> cfn;
    std::vector<uint32_t *> cqidx;  // per chunk: gather indices into the Q row (null: whole row)
    double *vscr = nullptr;
    size_t cap_vscr = 0;
    uint32_t ldv = 0;
    bool fused = false;  // this grid runs the fused forward kernel (no k_qrows)
    bool tall = false;   // this grid runs the reading kernel at kJitKblockTall threads
    uint32_t ncu = 0;    // the device's compute units (0: not asked yet)
    // wide path: per-chunk item factors, state-vector scratch, tables
    double *Pg = nullptr, *V = nullptr;
    size_t cap_pg = 0, cap_v = 0;
    uint32_t *np_d = nullptr, *udesc_w = nullptr;
    uint2 *mma_kt = nullptr, *mma_wplan = nullptr;
    uint32_t *mma_kbase = nullptr, *mma_desc = nullptr, *mma_dbase = nullptr;
    uint2 *mmt_kt = nullptr, *mmt_ktile = nullptr, *mmt_wplan = nullptr;  // k_fwd_mmt tables
    uint32_t *mmt_cidx = nullptr;
    // k_fwd_hs tables
    uint32_t *hs_kt = nullptr, *hs_cidx = nullptr, *hs_pbase = nullptr, *hs_dpos = nullptr, *hs_dbase = nullptr,
             *hs_pk = nullptr;
    uint2 *hs_ppos = nullptr, *hs_dpk = nullptr;
    uint4 *hs_wplan = nullptr;
    uint4 *hs_pass = nullptr;
    uint32_t wide_cb_items = 1, wide_cb_fwd = 1;  // c values per k_witems / k_fwd_wide launch
    std::vector<hipEvent_t> ev;  // kNumEv events per profiled run, reused
    std::vector<uint8_t> ev_mask;  // per profiled run: slots whose kernel was launched
    size_t ev_used = 0;          // event sets recorded since the last collect
};

}  // namespace

// Engine options (ABI 7, mdp_engine_create_opts): "NAME=VALUE" pairs
// separated by ';', ',' or white space.  They select among the engine's
// parity-tested kernel variants; the defaults are the
// measured best.  The library reads no tuning knob from the environment:
// mdp_engine_create is mdp_engine_create_opts with no options.  Names
// marked measurement-only exist in the diag build alone (-DMDP_DIAG_BUILD,
// libmidaspom_diag.so, used by scripts/): MDP_JIT_HACK's kernels do not
// store correct results, and phase stamps / occupancy hints are profiling
// aids.  An unknown name, or a measurement-only name in the default
// build, is MDP_EINVAL.
namespace {
const char *const kEngineOptNames[] = {
    "MDP_JIT", "MDP_FUSED", "MDP_FUSED_COLS", "MDP_EPL", "MDP_JIT_SLOTS", "MDP_JIT_WINDOW", "MDP_JIT_XCD",
    "MDP_JIT_EFAST", "MDP_QROWS_XCD", "MDP_FWD", "MDP_WIDE", "MDP_VSPLIT", "MDP_VLDS_EPL", "MDP_VLDS_MAXUSES",
    "MDP_JIT_CHUNK", "MDP_JIT_GATHER", "MDP_QGLOBAL", "MDP_FAST_LOG", "MDP_JIT_KBLOCK", "MDP_WIDE_CB",
    "MDP_JIT_CHECK", "MDP_JIT_DUMP", "MDP_JIT_THREADS", "MDP_JIT_VERBOSE", "MDP_JIT_SPLIT", "MDP_JIT_ROT",
    "MDP_WIDE_MMA", "MDP_HS_RADIX", "MDP_HS_WAVES"};
const char *const kDiagOptNames[] = {"MDP_DIAG", "MDP_JIT_HACK", "MDP_JIT_WPE", "MDP_HS_PROBE"};
#ifdef MDP_DIAG_BUILD
constexpr bool kDiagBuild = true;
#else
constexpr bool kDiagBuild = false;
#endif
}  // namespace

struct EngineOpts {
    std::map<std::string, std::string> kv;
    const char *get(const char *name) const
    {
        auto it = kv.find(name);
        return it == kv.end() ? nullptr : it->second.c_str();
    }
};

static int parse_engine_opts(const char *s, EngineOpts &o)
{
    o.kv.clear();
    if (!s) return MDP_OK;
    std::string cur;
    auto flush = [&]() -> int {
        if (cur.empty()) return MDP_OK;
        const size_t eq = cur.find('=');
        const std::string k = cur.substr(0, eq), v = eq == std::string::npos ? std::string("1") : cur.substr(eq + 1);
        cur.clear();
        bool known = false, diag = false;
        for (const char *n : kEngineOptNames) known |= k == n;
        for (const char *n : kDiagOptNames) diag |= k == n;
        if (diag && !kDiagBuild)
            return mdp_set_error(MDP_EINVAL, "option %s is measurement-only (libmidaspom_diag.so, -DMDP_DIAG_BUILD)",
                                 k.c_str());
        if (!known && !diag) return mdp_set_error(MDP_EINVAL, "unknown engine option '%s'", k.c_str());
        o.kv[k] = v;
        return MDP_OK;
    };
    for (const char *c = s;; ++c) {
        if (*c == 0 || *c == ';' || *c == ',' || *c == ' ' || *c == '\t' || *c == '\n') {
            const int rc = flush();
            if (rc) return rc;
            if (*c == 0) break;
        } else {
            cur += *c;
        }
    }
    return MDP_OK;
}

struct mdp_engine {
    uint32_t n = 0, tmax = 0, nvar = 0, nstates = 0, nextid = 0;
    uint32_t npairs = 0, nuses = 0, ncoef = 0, npmax = 1, variant = 0;
    uint32_t deg = 0;         // homogeneous transition degree D
    uint32_t maxA = 0;        // max |A| over uses
    int epl = kEPL;           // k_forward points per lane (MDP_EPL overrides: 1, 2, 4)
    bool fwd_lds = false;     // coefficient block staged in LDS (k_forward_lds)
    size_t fwd_lds_bytes = 0;
    bool lds_zpv = true;      // k_coefs stages Z/PV in LDS
    bool lds_part = true;     // k_coefs keeps subset partial sums in LDS
    bool diag = false;        // MDP_DIAG: record phase stamps
    bool jit = false;         // forward kernel specialised with hipRTC (spom_jit.cpp)
    bool wide = false;        // wide path (k_witems + k_wq + k_fwd_wide): npmax > 16 or MDP_WIDE=1
    bool qrows_xcd = true;    // k_qrows deals c ranges XCD-aware (MDP_QROWS_XCD=0: blockIdx order)
    double wide_flops_pt = 0; // its FP64 flops per grid point
    int jit_epl = 1;          // its grid points per lane (Q-row reading variant and chunks)
    uint32_t jit_kblock = kBlock;  // its threads per column
    // the fused variant's: 512 threads x 1 point per column by default (the
    // same 512 e rows per block as 256 x 2, so the grid shape is shared): with
    // one point per lane its 1 024-thread blocks fit 4 waves per SIMD, and the
    // per-column prologue runs over twice the threads (config 2: -2 to -3 %)
    int jit_epl_fused = 2;
    uint32_t jit_kblock_fused = kBlock;
    uint32_t jit_pro_fused = 2;
    bool jit_shape_env = false;  // MDP_EPL / MDP_JIT_KBLOCK set: one shape for both variants
    double jit_flops_pt = 0;  // its FP64 flops per grid point (counted by the generator)
    size_t ldQ = 0;           // per-c Q block (doubles, even) read by the JIT kernel
    std::vector<char> jit_code[3];  // forward kernel code objects [variant, as DevCtx::jit_fn], compiled on demand
    std::string jit_src[3];         // their sources (a cached object the runtime refuses is rebuilt)
    std::vector<std::string> chunk_src;
    std::vector<MdpJitPlan> chunks;               // > 1: the series runs as chunks of years
    std::vector<std::vector<char>> chunk_code;    // their code objects
    bool qglobal = false;     // Q rows built by k_zrows + k_witems + k_wq (k_qrows' tables exceed the LDS)
    int layout = MDP_LAYOUT_EC;  // mdp_engine_run's output layout (mdp_engine_set_layout)
    double cbound = 0.0;         // the per-c tables' |c| bound at least this (mdp_engine_set_cbound)
    int fused_mode = -1;            // MDP_FUSED: -1 auto, 0, 1
    MdpJitPlan jit_plan;
    // direct path (jit): k_qrows computes Pc[j][b] for the needed (j, b)
    // items, the forward kernel assembles Q from them
    uint32_t nj = 0, nitems = 0, ncoef_d = 0;
    size_t ldP = 0;
    std::vector<uint32_t> cj_bits, cj_item0, itemB, qstart, qitem, udesc_d, var_cols;
    std::vector<uint32_t> itemRow;  // row (j slot) of each item
    std::vector<uint2> qslot;       // k_qrows phase-3 lanes (build_direct_plan)
    std::vector<uint32_t> qlane;    // their groups' Pc slots, kQGroup a lane (nvar <= 8)
    std::vector<uint32_t> islot;    // k_qrows: each item's Pc slot (slots 0-15: zeros)
    uint32_t npl_slots = 0;         // k_qrows: Pc slots per c value
    uint32_t slot_conflicts = 0;    // k_qrows: extra gather cycles its slot colouring leaves (per c pair)
    uint32_t slot_store_conflicts = 0;  // and extra store-group conflicts
    // k_fwd_mma (wide years on the matrix cores): per year t its K entries
    // (k | |A_k| << 8 | m << 16 | valid << 31, padded to 4) from kbase[t],
    // and the Q-row slot of each (K entry, new state l) from gbase[t]
    bool mma = false;
    uint32_t mma_npm = 0;
    std::vector<uint2> mma_kt;  // per year its K entries: LDS byte offsets of the W rows, m, k
    std::vector<uint2> mma_wplan;  // per (year, wave) its work item (chunk range, column tile, slice)
    std::vector<uint32_t> mma_kbase, mma_desc, mma_dbase;
    uint32_t mma_ktmax = 16;
    // k_fwd_mmt (round 6, the default matrix-core forward: years of up to
    // 1 024 states): RT point tiles a block, per (year, tile) K lists, per
    // (year, wave) work items (build_mmt_plan)
    bool mmt = false;
    uint32_t mmt_rt = 0, mmt_rows = 0;
    std::vector<uint2> mmt_kt, mmt_ktile, mmt_wplan;
    std::vector<uint32_t> mmt_cidx;
    double mmt_flops_pt = 0;  // executed MFMA flops per grid point (padding included)
    // k_fwd_hs (round 6, through the hidden states: build_hs_plan): 2^hs_nb
    // cube positions, RT point tiles; per (year, tile) K lists of hidden
    // states and their item offsets, per year butterfly passes, the new
    // states' cube positions in tile order and free 16-row park blocks
    bool hs = false;
    uint32_t hs_rt = 0, hs_nb = 0, hs_nw = 16;
    uint32_t hs_probe = 0;  // MDP_HS_PROBE (timing probes only, wrong results): 1 skips v Pe, 2 U Pc
    std::vector<uint32_t> hs_kt, hs_cidx, hs_pbase, hs_dpos, hs_dbase, hs_pk;
    std::vector<uint2> hs_ppos, hs_dpk;
    std::vector<uint4> hs_wplan;
    std::vector<uint4> hs_pass;
    double hs_flops_pt = 0, hs_mfma_pt = 0;  // FP64 flops per grid point (padding included), of them MFMA
    std::vector<uint32_t> ystate;  // each year's states (short_state bits), year_off order
    uint32_t qslot_lglmax = 0;      // log2 of the widest lane segment
    std::vector<uint8_t> isvar;
    std::vector<double> Sj;  // [nj][n] colonisation sums of every column for each needed j
    std::string jit_log;
    size_t coef_lds = 0;      // k_coefs dynamic LDS bytes
    double prior0 = 1.0;
    std::vector<uint32_t> np, pairA, pairB, pairOff, use_pair, prog, udesc, pairPart0, partP, partK0;
    std::vector<DevCtx> devs;
    EngineOpts opts;          // mdp_engine_create_opts (variant selection; no environment reads)
    mutable std::set<std::string, std::less<>> launched;  // kernel instantiations launched so far (mdp_engine_launched)
    mutable std::mutex launched_mu;                         // engines may be driven from several host threads
    int profiling = 0;
    double last_ms[3] = {0, 0, 0};  // mean per run over the last collected runs
    int nlast = 0;
    uint64_t runs_collected = 0;
};

namespace {

// The forward kernels' output strides: log L of point (ie, ic) at
// out[ie * se + ic * sc] -- [e][c] rows (se = ld, sc = 1) or [c][e] columns
// (se = 1, sc = ld); every forward kernel takes both.  Passed explicitly down
// every launch path: only mdp_engine_run / mdp_engine_time_kernels honour the
// engine's layout (mdp_engine_set_layout); mdp_loglik_grid always fills its
// device slab in [e][c] (its host contract).
struct OutStrides {
    uint32_t se, sc;
};
inline OutStrides layout_strides(int layout, uint32_t ld)
{
    return layout == MDP_LAYOUT_CE ? OutStrides{1u, ld} : OutStrides{ld, 1u};
}

// record a launched kernel instantiation ("k_qrows<16,0,2>", ...)
void note_launch(const mdp_engine *eng, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
void note_launch(const mdp_engine *eng, const char *fmt, ...)
{
    char b[96];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(b, sizeof b, fmt, ap);
    va_end(ap);
    // look up before inserting: the hot path re-launches the same kernels, so
    // after the first launch of each this allocates nothing
    std::lock_guard<std::mutex> lk(eng->launched_mu);
    if (eng->launched.find(b) == eng->launched.end()) eng->launched.emplace(b);
}

constexpr int kDegBuckets[] = {4, 8, 16, 24};

int select_variant(mdp_engine *eng)
{
    uint32_t np = 0;
    for (uint32_t b : {1u, 2u, 4u, 8u, 16u})
        if (eng->npmax <= b) { np = b; break; }
    // a year with more than 16 states (over 4 missing patches) exceeds the
    // register-resident forward kernels: the wide path takes the problem
    if (!np) eng->wide = true;
    uint32_t deg = 0;
    for (int b : kDegBuckets)
        if (eng->maxA <= (uint32_t)b) { deg = (uint32_t)b; break; }
    if (!deg) return mdp_set_error(MDP_EUNSUPPORTED, "%u occupied patches in one state (max %d)", eng->maxA, kMaxDeg);
    eng->deg = deg;
    eng->variant = eng->wide ? 20000u + deg : np * 100 + deg;
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
    if (const char *wv = eng->opts.get("MDP_WIDE")) eng->wide = atoi(wv) != 0;
    eng->np.resize(p->tmax);
    eng->npmax = 1;
    for (uint32_t t = 0; t < p->tmax; ++t) {
        eng->np[t] = p->year_off[t + 1] - p->year_off[t];
        eng->npmax = std::max(eng->npmax, eng->np[t]);
    }
    eng->ystate.clear();
    for (uint32_t i = 0; i < p->year_off[p->tmax]; ++i)
        eng->ystate.push_back(p->year_ids[i] < p->nextid ? p->short_state[p->year_ids[i]] : ~0u);
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
    // k_coefs subset parts (pair, first subset index), and per-use descriptors
    for (uint32_t pi = 0; pi < eng->pairA.size(); ++pi) {
        const uint32_t nX = (uint32_t)__builtin_popcount(eng->pairA[pi] & eng->pairB[pi]);
        eng->pairPart0.push_back((uint32_t)eng->partP.size());
        for (uint32_t k0 = 0; k0 < (1u << nX); k0 += kSubPart) {
            eng->partP.push_back(pi);
            eng->partK0.push_back(k0);
        }
    }
    eng->pairPart0.push_back((uint32_t)eng->partP.size());
    if (off > kOffMask) return mdp_set_error(MDP_EUNSUPPORTED, "too many transition coefficients");
    for (uint32_t pi : eng->use_pair) {
        const uint32_t A = eng->pairA[pi], B = eng->pairB[pi];
        const uint32_t nA = (uint32_t)__builtin_popcount(A), nX = (uint32_t)__builtin_popcount(A & B);
        eng->udesc.push_back(eng->pairOff[pi] | (nX << kOffBits) | (nA << 27));
    }
    eng->npairs = (uint32_t)eng->pairA.size();
    eng->nuses = (uint32_t)eng->use_pair.size();
    eng->ncoef = off;
    int rc = select_variant(eng);
    if (rc) return rc;
    if (eng->wide) return MDP_OK;  // no step program / k_coefs plan: build_wide_plan
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
    // k_coefs LDS plan: [Z/PV block] [part partials] [Q] [binomials]; the
    // partials spill to a global scratch when they do not fit
    const size_t zbytes = (size_t)(eng->nvar + 1) * eng->nstates * sizeof(double);
    const size_t pbytes = (size_t)eng->partP.size() * (eng->nvar + 1) * sizeof(double);
    const size_t qbytes = ((size_t)eng->ncoef + (size_t)(kMaxDeg + 1) * (kMaxDeg + 1)) * sizeof(double);
    if (zbytes + pbytes + qbytes <= kLdsBudget) {
        eng->lds_zpv = eng->lds_part = true;
        eng->coef_lds = zbytes + pbytes + qbytes;
    } else if (pbytes + qbytes <= kLdsBudget) {
        eng->lds_zpv = false;
        eng->lds_part = true;
        eng->coef_lds = pbytes + qbytes;
    } else if (qbytes <= kLdsBudget) {
        eng->lds_zpv = eng->lds_part = false;
        eng->coef_lds = qbytes;
    } else {
        return mdp_set_error(MDP_EUNSUPPORTED, "%u transition coefficients exceed the LDS budget",
                             eng->ncoef);
    }
    return MDP_OK;
}

// Direct-path plan.  Transitions that share X = A & B and the target state B
// share Q; each (X, B) group needs Pc[j][B] for every j <= X.  Items are the
// distinct (j, B), numbered by j ascending then B ascending; qstart / qitem
// list, for every Q entry (group, m), its items with |j| = m in ascending j.
int build_direct_plan(mdp_engine *eng, const mdp_problem *p)
{
    std::map<uint64_t, uint32_t> group;  // (X, B) -> Q offset
    std::vector<std::pair<uint32_t, uint32_t>> groups;
    std::vector<uint32_t> pair_group(eng->pairA.size());
    uint32_t off = 0;
    std::vector<uint32_t> goff;
    for (size_t pi = 0; pi < eng->pairA.size(); ++pi) {
        const uint32_t B = eng->pairB[pi], X = eng->pairA[pi] & B;
        const uint64_t key = ((uint64_t)X << 32) | B;
        auto it = group.find(key);
        if (it == group.end()) {
            it = group.emplace(key, (uint32_t)groups.size()).first;
            groups.push_back({X, B});
            // even start: the forward kernels read a group's coefficients
            // pairwise as 16-byte aligned ds_read_b128 (an unaligned pair
            // becomes a ds_read2_b64, twice the LDS cycles per byte)
            off = (off + 1u) & ~1u;
            goff.push_back(off);
            off += (uint32_t)__builtin_popcount(X) + 1u;
        }
        pair_group[pi] = it->second;
    }
    if (off > kOffMask) return mdp_set_error(MDP_EUNSUPPORTED, "too many transition coefficients");
    eng->ncoef_d = off;
    std::map<uint32_t, std::vector<uint32_t>> jb;  // j -> states B (sorted, unique)
    auto for_subsets = [](uint32_t X, auto &&fn) {  // ascending j <= X
        const uint32_t nX = (uint32_t)__builtin_popcount(X);
        for (uint32_t k = 0; k < (1u << nX); ++k) {
            uint32_t j = 0, xs = X;
            for (uint32_t i = 0; i < nX; ++i) {
                const uint32_t low = xs & (0u - xs);
                if ((k >> i) & 1u) j |= low;
                xs ^= low;
            }
            fn(j);
        }
    };
    for (auto &g : groups) for_subsets(g.first, [&](uint32_t j) { jb[j].push_back(g.second); });
    std::map<uint64_t, uint32_t> item;  // (j, B) -> item
    eng->cj_bits.clear();
    eng->cj_item0.clear();
    eng->itemB.clear();
    for (auto &kv : jb) {
        auto &v = kv.second;
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
        eng->cj_bits.push_back(kv.first);
        eng->cj_item0.push_back((uint32_t)eng->itemB.size());
        for (uint32_t B : v) {
            item.emplace(((uint64_t)kv.first << 32) | B, (uint32_t)eng->itemB.size());
            eng->itemB.push_back(B);
        }
    }
    eng->cj_item0.push_back((uint32_t)eng->itemB.size());
    eng->nj = (uint32_t)eng->cj_bits.size();
    if (eng->nj > 0xffffu) return mdp_set_error(MDP_EUNSUPPORTED, "%u hidden-state rows (direct path max 65535)", eng->nj);
    eng->itemRow.assign(eng->itemB.size(), 0u);
    for (uint32_t js = 0; js < eng->nj; ++js)
        for (uint32_t i = eng->cj_item0[js]; i < eng->cj_item0[js + 1]; ++i) eng->itemRow[i] = js;
    eng->nitems = (uint32_t)eng->itemB.size();
    eng->ldP = ((size_t)eng->nitems + 1) & ~(size_t)1;
    eng->qstart.assign(1, 0u);
    eng->qitem.clear();
    for (auto &g : groups) {
        const uint32_t nX = (uint32_t)__builtin_popcount(g.first);
        if ((eng->qstart.size() - 1) & 1u) eng->qstart.push_back((uint32_t)eng->qitem.size());  // pad slot
        for (uint32_t m = 0; m <= nX; ++m) {
            for_subsets(g.first, [&](uint32_t j) {
                if ((uint32_t)__builtin_popcount(j) == m)
                    eng->qitem.push_back(item.at(((uint64_t)j << 32) | g.second));
            });
            eng->qstart.push_back((uint32_t)eng->qitem.size());
        }
    }
    // k_qrows' phase-3 lane table (the canonical Q-sum order, kQGroup): per
    // entry q < ldQ an aligned segment of L = min(P, kQLanesMax) lanes, P =
    // its group count rounded up to a power of two, each lane 2^G = P / L
    // groups; segments packed largest first, so each is aligned and lies in
    // one wave; padded to whole waves
    {
        const size_t ldq = ((size_t)off + 1) & ~(size_t)1;
        struct Ent { uint32_t lgL, lgG, q; };
        std::vector<Ent> ents;
        for (uint32_t q = 0; q < ldq; ++q) {
            const uint32_t n = q + 1 < eng->qstart.size() ? eng->qstart[q + 1] - eng->qstart[q] : 0u;
            const uint32_t ng = std::max<uint32_t>(1u, (n + kQGroup - 1) / kQGroup);
            uint32_t lgP = 0;
            while ((1u << lgP) < ng) ++lgP;
            uint32_t lgL = 0;
            while ((1u << lgL) < kQLanesMax && lgL < lgP) ++lgL;
            if (lgP - lgL >= (uint32_t)kQLevelsRows)
                return mdp_set_error(MDP_EUNSUPPORTED, "a Q entry of %u items (k_qrows' lane table)", n);
            ents.push_back({lgL, lgP - lgL, q});
        }
        std::stable_sort(ents.begin(), ents.end(), [](const Ent &x, const Ent &y) { return x.lgL > y.lgL; });
        eng->qslot.clear();
        eng->qslot_lglmax = ents.empty() ? 0u : ents[0].lgL;
        for (const Ent &en : ents)
            for (uint32_t le = 0; le < (1u << en.lgL); ++le)
                eng->qslot.push_back(make_uint2(en.q, le | (en.lgL << 8) | (en.lgG << 12)));
        while (eng->qslot.size() % 64) eng->qslot.push_back(make_uint2(0xffffffffu, 0u));
        // nvar <= 8 (one group per lane): each lane's kQGroup items, nitems
        // past its entry; at least 64 lanes
        const uint32_t ni = eng->nitems;
        eng->qlane.assign(std::max<size_t>(eng->qslot.size(), 64) * kQGroup, ni);
        if (eng->nvar <= 8)
            for (size_t sl = 0; sl < eng->qslot.size(); ++sl) {
                const uint32_t q = eng->qslot[sl].x, le = eng->qslot[sl].y & 0xffu;
                if ((size_t)q + 1 >= eng->qstart.size()) continue;  // padding lanes: q = ~0
                const uint32_t j0 = eng->qstart[q] + le * kQGroup, i1 = eng->qstart[q + 1];
                for (uint32_t u = 0; u < kQGroup && j0 + u < i1; ++u) eng->qlane[sl * kQGroup + u] = eng->qitem[j0 + u];
            }
        // Pc slots (16 bytes per slot and c pair in LDS).  Phase 3 gathers
        // item u of every lane in one ds_read_b128, serviced in four 16-lane
        // groups, conflict-free when a group's slots differ mod 16; phase 2
        // stores eight consecutive items per 8-lane group of a
        // ds_write_b128, conflict-free when they differ mod 8.  The items are
        // coloured (colour = slot mod 16) greedily under both rules, the
        // least-used allowed colour first; slots 0-15 hold zeros, and each
        // group's padding takes the zero slot of a colour none of its items
        // has.  nvar > 8 (CSR path): slot = item + 16.
        eng->islot.resize(ni);
        for (uint32_t it = 0; it < ni; ++it) eng->islot[it] = it + 16;
        eng->npl_slots = ni + 16;
        if (eng->nvar <= 8) {
            auto lgroup = [](uint32_t l) -> uint32_t {  // ds_read_b128 lane groups
                const uint32_t h = l & 31u;
                const uint32_t g = (h < 4 || (h >= 12 && h < 16) || (h >= 20 && h < 28)) ? 0u : 1u;
                return g + (l >= 32 ? 2u : 0u);
            };
            const size_t nl = eng->qslot.size();
            std::vector<std::vector<uint32_t>> grp;  // per (wave, u, lane group): its items
            for (size_t w0 = 0; w0 < nl; w0 += 64)
                for (uint32_t u = 0; u < kQGroup; ++u) {
                    std::vector<uint32_t> g4[4];
                    for (uint32_t l = 0; l < 64 && w0 + l < nl; ++l) {
                        const uint32_t it = eng->qlane[(w0 + l) * kQGroup + u];
                        if (it < ni) g4[lgroup(l)].push_back(it);
                    }
                    for (auto &g : g4) {
                        std::sort(g.begin(), g.end());
                        g.erase(std::unique(g.begin(), g.end()), g.end());
                        grp.push_back(std::move(g));
                    }
                }
            std::vector<std::vector<uint32_t>> ig(ni);
            for (uint32_t gi = 0; gi < grp.size(); ++gi)
                for (uint32_t it : grp[gi]) ig[it].push_back(gi);
            std::vector<int> col(ni, -1);
            uint32_t cnt[16] = {};
            for (uint32_t it = 0; it < ni; ++it) {
                uint32_t forb = 0;
                for (uint32_t gi : ig[it])
                    for (uint32_t o : grp[gi])
                        if (col[o] >= 0) forb |= 1u << col[o];
                for (uint32_t o = it & ~7u; o < (it | 7u) + 1 && o < ni; ++o)  // phase 2's store group
                    if (o != it && col[o] >= 0) forb |= 0x101u << (col[o] & 7);
                int best = -1;
                for (int pass = 0; pass < 2 && best < 0; ++pass)
                    for (int cc = 0; cc < 16; ++cc)
                        if ((pass || !((forb >> cc) & 1u)) && (best < 0 || cnt[cc] < cnt[best])) best = cc;
                col[it] = best;
                ++cnt[best];
            }
            // min-conflicts repair: move an item to the colour its groups use
            // least while that lowers its own conflicts (each move lowers the
            // total, which is symmetric in the pairs), a few sweeps.  A gather
            // conflict costs a cycle per group; a store conflict only about a
            // quarter of one (a ds_write_b128's transfer, 13 cycles, hides all
            // but 3 of the 16 array cycles of a 2-way conflict): weights 4 : 1
            for (int sweep = 0; sweep < 16; ++sweep) {
                bool moved = false;
                for (uint32_t it = 0; it < ni; ++it) {
                    uint32_t cost[16] = {};
                    for (uint32_t gi : ig[it])
                        for (uint32_t o : grp[gi])
                            if (o != it) cost[col[o]] += 4;
                    for (uint32_t o = it & ~7u; o < (it | 7u) + 1 && o < ni; ++o)
                        if (o != it) {
                            ++cost[col[o] & 7];
                            ++cost[(col[o] & 7) + 8];
                        }
                    int best = col[it];
                    for (int cc = 0; cc < 16; ++cc)
                        if (cost[cc] < cost[best] || (cost[cc] == cost[best] && cnt[cc] + 1 < cnt[best])) best = cc;
                    if (best != col[it]) {
                        --cnt[col[it]];
                        ++cnt[best];
                        col[it] = best;
                        moved = true;
                    }
                }
                if (!moved) break;
            }
            uint32_t next[16];
            for (uint32_t cc = 0; cc < 16; ++cc) next[cc] = 16 + cc;
            uint32_t top = 16;
            for (uint32_t it = 0; it < ni; ++it) {
                eng->islot[it] = next[col[it]];
                next[col[it]] += 16;
                top = std::max(top, eng->islot[it] + 1);
            }
            eng->npl_slots = top;
            // what the colouring leaves: per phase-3 group the extra cycles of
            // its busiest residue, per phase-2 store group those mod 8
            uint32_t extra = 0, sextra = 0;
            for (const auto &g : grp) {
                uint32_t m[16] = {};
                for (uint32_t it : g) ++m[eng->islot[it] & 15u];
                extra += *std::max_element(m, m + 16) - (g.empty() ? 0u : 1u);
            }
            for (uint32_t g0 = 0; g0 < ni; g0 += 8) {
                uint32_t m[8] = {};
                for (uint32_t it = g0; it < std::min(ni, g0 + 8); ++it) ++m[eng->islot[it] & 7u];
                sextra += *std::max_element(m, m + 8) - 1u;
            }
            eng->slot_conflicts = extra;
            eng->slot_store_conflicts = sextra;
            // the lanes' slots; each (wave, u, lane group)'s padding on a free colour
            for (size_t w0 = 0; w0 < std::max<size_t>(nl, 64); w0 += 64)
                for (uint32_t u = 0; u < kQGroup; ++u) {
                    uint32_t used[4] = {};
                    for (uint32_t l = 0; l < 64; ++l) {
                        const uint32_t it = eng->qlane[(w0 + l) * kQGroup + u];
                        if (it < ni) used[lgroup(l)] |= 1u << (eng->islot[it] & 15u);
                    }
                    for (uint32_t l = 0; l < 64; ++l) {
                        uint32_t &x = eng->qlane[(w0 + l) * kQGroup + u];
                        if (x < ni) {
                            x = eng->islot[x];
                        } else {
                            const uint32_t fr = ~used[lgroup(l)] & 0xffffu;
                            x = fr ? (uint32_t)__builtin_ctz(fr) : 0u;
                        }
                    }
                }
        }
    }
    eng->udesc_d.clear();
    for (uint32_t pi : eng->use_pair) {
        const uint32_t A = eng->pairA[pi], B = eng->pairB[pi];
        const uint32_t nA = (uint32_t)__builtin_popcount(A), nX = (uint32_t)__builtin_popcount(A & B);
        eng->udesc_d.push_back(goff[pair_group[pi]] | (nX << kOffBits) | (nA << 27));
    }
    // colonisation sums S[j][k] = sum over var columns l in j (ascending),
    // l != k, of M[l][k] -- the reference's per-point sum (:350-357) with its
    // zero terms dropped, in its order
    const uint32_t n = p->n, nvar = p->nvar;
    eng->var_cols.assign(p->var_cols, p->var_cols + nvar);
    eng->isvar.assign(n, 0);
    for (uint32_t b = 0; b < nvar; ++b) eng->isvar[p->var_cols[b]] = 1;
    eng->Sj.assign((size_t)eng->nj * n, 0.0);
    for (uint32_t js = 0; js < eng->nj; ++js) {
        const uint32_t j = eng->cj_bits[js];
        for (uint32_t k = 0; k < n; ++k) {
            double acc = 0.0;
            for (uint32_t b = 0; b < nvar; ++b) {
                const uint32_t col = p->var_cols[b];
                if (((j >> (nvar - 1 - b)) & 1u) && col != k) acc += p->M[(size_t)col * n + k];
            }
            eng->Sj[(size_t)js * n + k] = acc;
        }
    }
    return MDP_OK;
}

// Wide-path plan: the direct plan's groups, items and per-use descriptors,
// plus the FP64 work per grid point of k_fwd_wide (every use a (nX+1)-term
// dot product with a weight multiply per term, one FMA into the state
// vector; the per-lane power tables; the final prior sum).
// k_fwd_mma: two state buffers and the power tables of the block's points,
// and (LDS staging) three years' K entries
size_t mma_lds(const mdp_engine *eng)
{
    const uint32_t npm = eng->mma_npm;
    return (2 * (size_t)mma_rows(npm) * mma_pts(npm) + 2 * ((size_t)eng->maxA + 1) * mma_ps(npm)) * sizeof(double) +
           0;
}

// the k_fwd_mma instantiation of the engine's plan
const void *mma_kernel(const mdp_engine *eng)
{
    if (eng->mma_npm == 64) return (const void *)k_fwd_mma<64>;
    if (eng->mma_npm == 128) return (const void *)k_fwd_mma<128>;
    return (const void *)k_fwd_mma<256>;
}

// the device's LDS per workgroup (the current device; 160 KiB on gfx950)
size_t device_lds_max()
{
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) == hipSuccess && v > 0)
        return (size_t)v;
    return 160 * 1024;
}

// k_fwd_mmt: the state buffer and the power tables of the block's points
// k_fwd_mmt's shapes by the largest year: RT point tiles, state rows, two buffers
struct MmtShape {
    uint32_t rt, rows;
    bool db;
};
// (measured, profiles/r06/wide: years of up to 128 states run 25 % faster on
// <4, 128, 2buf> than on <2, 256, 1buf>; a 256-state problem 6 % faster on
// one buffer than on <2, 256, 2buf>)
inline MmtShape mmt_shape(const mdp_engine *eng)
{
    const uint32_t npmax = eng->npmax;
    if (npmax <= 128) return {4u, 128u, true};
    if (npmax <= 256) return {2u, 256u, false};
    if (npmax <= 512) return {2u, 512u, false};
    return {1u, 1024u, false};
}

size_t mmt_lds(const mdp_engine *eng)
{
    const MmtShape sh = mmt_shape(eng);
    return ((sh.db ? 2 : 1) * (size_t)sh.rows * mmt_pts(sh.rt) + 2 * ((size_t)eng->maxA + 1) * mmt_ps(sh.rt)) *
           sizeof(double);
}

const void *mmt_kernel(const mdp_engine *eng)
{
    if (eng->mmt_rows == 128) return (const void *)k_fwd_mmt<4, 128, true>;
    if (eng->mmt_rows == 256) return (const void *)k_fwd_mmt<2, 256, false>;
    if (eng->mmt_rows == 512) return (const void *)k_fwd_mmt<2, 512, false>;
    return (const void *)k_fwd_mmt<1, 1024, false>;
}

// per (year, wave) work items over a year's column tiles of nch[tile]
// pipeline chunks each (k_fwd_mmt, k_fwd_hs): more than 16 tiles are dealt
// longest list first to the least-loaded wave (up to tmaxit each); up to 16
// give every tile a wave and the spare waves to the tiles whose slices are
// longest (at least two chunks each; slices past the first `inplace` of a
// tile park their partials, `room` 16-row blocks at most)
void plan_waves(const std::vector<uint32_t> &nch, uint32_t tmaxit, uint32_t inplace, uint32_t room, uint2 *wp,
                uint32_t nw = 16)
{
    const uint32_t ncol = (uint32_t)nch.size();
    if (ncol <= nw) {
        // waves per tile: one each, the rest to the tile whose slices
        // are longest (each slice at least two chunks; the parked
        // partials -- every slice past the first `inplace` of a tile --
        // within the buffer's rows past the year's tiles)
        std::vector<uint32_t> w(ncol, 1);
        uint32_t parked = 0;
        for (uint32_t spare = nw - ncol; spare; --spare) {
            uint32_t best = ncol;
            for (uint32_t i = 0; i < ncol; ++i)
                if (nch[i] / (w[i] + 1) >= 2 && (w[i] + 1 <= inplace || parked < room) &&
                    (best == ncol || nch[i] * w[best] > nch[best] * w[i]))
                    best = i;
            if (best == ncol) break;
            if (++w[best] > inplace) ++parked;
        }
        const uint32_t split = *std::max_element(w.begin(), w.end()) > 1 ? 1u : 0u;
        for (uint32_t wv = 0; wv < nw; ++wv)
            for (uint32_t i = 0; i < tmaxit; ++i) wp[wv * tmaxit + i] = make_uint2(0u, split << 22);
        uint32_t wv = 0, pbase = 0;
        for (uint32_t tile = 0; tile < ncol; ++tile) {
            for (uint32_t ks = 0; ks < w[tile]; ++ks, ++wv) {
                const uint32_t cb = nch[tile] * ks / w[tile], ce = nch[tile] * (ks + 1) / w[tile];
                wp[wv * tmaxit] = make_uint2(cb | ce << 16, tile | ks << 8 | w[tile] << 12 | pbase << 17 |
                                                               split << 22 | 1u << 24);
            }
            pbase += w[tile] > inplace ? w[tile] - inplace : 0;
        }
    } else {
        std::vector<uint32_t> order(ncol), cnt(nw, 0);
        std::vector<uint64_t> load(nw, 0);
        for (uint32_t i = 0; i < ncol; ++i) order[i] = i;
        std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return nch[x] > nch[y]; });
        for (uint32_t wv = 0; wv < nw; ++wv)
            for (uint32_t i = 0; i < tmaxit; ++i) wp[wv * tmaxit + i] = make_uint2(0u, 0u);
        for (uint32_t tile : order) {
            uint32_t best = nw;
            for (uint32_t wv = 0; wv < nw; ++wv)
                if (cnt[wv] < tmaxit && (best == nw || load[wv] < load[best])) best = wv;
            wp[best * tmaxit + cnt[best]++] = make_uint2(nch[tile] << 16, tile | 1u << 12 | 1u << 24);
            load[best] += nch[tile];
        }
    }
}

// k_fwd_mmt's tables (c-independent): years of at most 1 024 states.
//  * per (year, column tile) its K entries: every source k with m = 0 ..
//    the largest nX over the tile's new states (the rest of m <= |A_k| would
//    meet only zero slots), padded to whole pipeline chunks; and per K entry
//    and new state l of the tile, the byte offset in the Q row of Q_kl[m]
//    (the zero slot where m > nX_kl, for padded states and padded entries)
//    -- 64 bytes per entry, so the kernel's gathers need no lookup;
//  * per (year, wave) up to ROWS / 256 work items: tiles of years of more
//    than 16 tiles dealt longest list first to the least-loaded wave;
//    smaller years give every tile a wave and the spare waves to the tiles
//    with the longest lists, each tile's list split into as many slices
//    (at least two chunks each).
void build_mmt_plan(mdp_engine *eng)
{
    if (eng->npmax > 1024 || eng->maxA > 24 || eng->tmax < 2) return;
    const MmtShape shp = mmt_shape(eng);
    const uint32_t rows = shp.rows, rt = shp.rt, pts = mmt_pts(rt), ps = mmt_ps(rt);
    const uint32_t tmaxit = rows > 256 ? rows / 256 : 1, cw = 4 * mmt_u(rt), inplace = shp.db ? 2u : 1u;
    const uint32_t none = (uint32_t)eng->ncoef_d;
    if (none > kOffMask) return;
    eng->mmt_rt = rt;
    eng->mmt_rows = rows;
    eng->mmt_kt.clear();
    eng->mmt_cidx.clear();
    eng->mmt_ktile.assign((size_t)(eng->tmax + 1) * kMmtMaxTiles, make_uint2(0u, 1u));
    eng->mmt_wplan.assign((size_t)(eng->tmax + 1) * 16 * tmaxit, make_uint2(0u, 0u));
    double fl = 0.0;
    size_t ub = 0;
    for (uint32_t t = 1; t < eng->tmax; ++t) {
        const uint32_t npp = eng->np[t - 1], npc = eng->np[t], ncol = (npc + 15) / 16;
        const uint32_t *ud = eng->udesc_d.data() + ub;  // ud[l * npp + k]
        std::vector<uint32_t> nch(ncol);
        for (uint32_t tile = 0; tile < ncol; ++tile) {
            const size_t start = eng->mmt_kt.size();
            const uint32_t l1 = std::min(16 * tile + 16, npc);
            for (uint32_t k = 0; k < npp; ++k) {
                const uint32_t a = ud[k] >> 27;  // |A_k|
                uint32_t mx = 0;
                for (uint32_t l = 16 * tile; l < l1; ++l) mx = std::max(mx, (ud[(size_t)l * npp + k] >> kOffBits) & 31u);
                for (uint32_t m = 0; m <= mx; ++m) {  // V row k, y^m row, x^(a-m) row (bytes); m; k
                    eng->mmt_kt.push_back(make_uint2((k * pts * 8u) | ((m * ps * 8u) << 18),
                                                     ((a - m) * ps * 8u) | (m << 16) | (k << 21)));
                    for (uint32_t l = 16 * tile; l < 16 * tile + 16; ++l) {
                        uint32_t o = none;
                        if (l < npc) {
                            const uint32_t dsc = ud[(size_t)l * npp + k];
                            if (m <= ((dsc >> kOffBits) & 31u)) o = (dsc & kOffMask) + m;
                        }
                        eng->mmt_cidx.push_back(o * 8u);
                    }
                }
            }
            while ((eng->mmt_kt.size() - start) % cw) {
                eng->mmt_kt.push_back(make_uint2(0u, npp << 21));
                for (uint32_t l = 0; l < 16; ++l) eng->mmt_cidx.push_back(none * 8u);
            }
            nch[tile] = (uint32_t)((eng->mmt_kt.size() - start) / cw);
            eng->mmt_ktile[(size_t)t * kMmtMaxTiles + tile] = make_uint2((uint32_t)start, nch[tile]);
            fl += 2.0 * 16.0 * (double)(eng->mmt_kt.size() - start);
        }
        plan_waves(nch, tmaxit, inplace, (rows - ncol * 16) / 16, eng->mmt_wplan.data() + (size_t)t * 16 * tmaxit);
        ub += (size_t)npp * npc;
    }
    eng->mmt_flops_pt = fl + 2.0 * (eng->maxA + 1) + (double)eng->np[eng->tmax - 1];
    // (the offsets' table is the plan's largest: 64 bytes per K entry)
    eng->mmt = mmt_lds(eng) <= device_lds_max() && eng->mmt_kt.size() < (1u << 26) && (size_t)none * 8u < 0xffffffffu;
    if (!eng->mmt) {
        eng->mmt_kt.clear();
        eng->mmt_cidx.clear();
    }
}

// k_fwd_hs: the cube of the block's points (128 KiB for each shape)
size_t hs_lds(const mdp_engine *eng)
{
    return (((size_t)1 << eng->hs_nb) + eng->hs_nb + 1) * mmt_pts(eng->hs_rt) * sizeof(double);  // + y^k table
}

const void *hs_kernel(const mdp_engine *eng)
{
    if (eng->hs_nb == 8) return eng->hs_nw == 8 ? (const void *)k_fwd_hs<2, 8, 8> : (const void *)k_fwd_hs<4, 8, 16>;
    if (eng->hs_nb == 9) return (const void *)k_fwd_hs<2, 9, 16>;
    return (const void *)k_fwd_hs<1, 10, 16>;
}

// k_fwd_hs's tables (c-independent; nvar <= 10, years of at most 1 024
// states).  Per year t >= 1:
//  * butterfly passes over W = the bits of year t - 1's states, up to
//    kHsRadix patches a pass: first the patches set in no hidden state the
//    year's products read, then greedily the one adding the fewest new cube
//    positions; a pass lists its cosets (g, the masks of the positions it
//    reads and writes: only those whose value still reaches a hidden state
//    the products read).  After the passes every such j holds U[j];
//  * the year's states ordered by (B & W, B), so a tile's 16 states share
//    their reachable hidden states; per tile K = the j in that down-closure
//    below some state of the tile, ascending, padded to whole pipeline
//    chunks (row 0, C = 0), and per (K entry, state) the byte offset of the
//    item Pc[j][B] in the column's Pg row (its zero slot, nitems, for j not
//    below B, padded states and padded entries);
//  * the states' cube positions in tile order (~0: padding), the free 16-row
//    park blocks (no state of the year in them), the wave plan.
// Year 0's positions head dpos.  Refused (hs = false: k_fwd_mmt runs) for a
// year with a repeated state or an item the direct plan lacks.
void build_hs_plan(mdp_engine *eng)
{
    eng->hs = false;
    if (eng->nvar > 10 || eng->tmax < 2 || eng->npmax > 1024 || eng->ystate.size() < eng->tmax) return;
    const uint32_t nb = std::max<uint32_t>(8u, eng->nvar);
    // waves a block (MDP_HS_WAVES): 8 for 8 variable patches (32 points, a
    // 64 KiB cube: two blocks a CU, whose phases overlap; measured 5 % faster
    // on the 256-state series, equal on the 128-state one, profiles/r06/hs),
    // else 16
    uint32_t nw = nb == 8 ? 8u : 16u;
    if (const char *wv = eng->opts.get("MDP_HS_WAVES")) nw = atoi(wv) == 8 && nb == 8 ? 8u : 16u;
    const uint32_t rt = nb == 8 ? (nw == 8 ? 2u : 4u) : nb == 9 ? 2u : 1u, pts = mmt_pts(rt);
    const uint32_t ncube = 1u << nb, tmaxit = ncube / 16 > nw ? ncube / 16 / nw : 1u, cw = 4 * mmt_u(rt);
    const uint32_t zero = eng->nitems;  // the Pg row's zero slot
    if ((uint64_t)zero * 8u >= 0xffffffffull) return;
    // patches per v Pe pass (MDP_HS_RADIX, 1 .. kHsRadix; default 4, the
    // measured best: profiles/r06/hs -- 1 024 cosets x points fill the block
    // in one sweep; 5 left half the threads idle on 1 024-state years)
    uint32_t radix = kHsRadix;
    if (const char *rv = eng->opts.get("MDP_HS_RADIX")) radix = std::min<uint32_t>(kHsRadix, std::max(1, atoi(rv)));
    std::unordered_map<uint64_t, uint32_t> item;  // (j, B) -> item
    for (uint32_t js = 0; js < eng->nj; ++js)
        for (uint32_t i = eng->cj_item0[js]; i < eng->cj_item0[js + 1]; ++i)
            item.emplace(((uint64_t)eng->cj_bits[js] << 32) | eng->itemB[i], i);
    std::vector<uint32_t> yoff(eng->tmax + 1, 0);
    for (uint32_t t = 0; t < eng->tmax; ++t) yoff[t + 1] = yoff[t] + eng->np[t];
    auto st = [&](uint32_t t, uint32_t l) { return eng->ystate[yoff[t] + l]; };
    eng->hs_kt.clear();
    eng->hs_cidx.clear();
    eng->hs_pass.clear();
    eng->hs_ppos.clear();
    eng->hs_dpos.clear();
    std::vector<uint2> ktile(kMmtMaxTiles), wtmp(nw * tmaxit);
    eng->hs_wplan.assign((size_t)(eng->tmax + 1) * nw * tmaxit, make_uint4(0u, 0u, 0u, 1u));
    eng->hs_pk.assign((size_t)(eng->tmax + 1) * 16, 0u);
    eng->hs_pbase.assign(eng->tmax + 1, 0u);
    eng->hs_dbase.assign(eng->tmax + 1, 0u);
    std::vector<uint8_t> seen(ncube, 0);
    auto distinct = [&](uint32_t t) {
        bool ok = true;
        for (uint32_t l = 0; l < eng->np[t]; ++l) {
            const uint32_t b = st(t, l);
            if (b >= ncube || seen[b]) ok = false;
            else seen[b] = 1;
        }
        for (uint32_t l = 0; l < eng->np[t]; ++l)
            if (st(t, l) < ncube) seen[st(t, l)] = 0;
        return ok;
    };
    if (!distinct(0)) return;
    for (uint32_t l = 0; l < (eng->np[0] + 15) / 16 * 16; ++l) eng->hs_dpos.push_back(l < eng->np[0] ? st(0, l) : ~0u);
    double fb = 0.0, fm = 0.0;
    std::vector<uint8_t> live(ncube);
    std::vector<uint32_t> lv;
    for (uint32_t t = 1; t < eng->tmax; ++t) {
        const uint32_t npp = eng->np[t - 1], npc = eng->np[t], ncol = (npc + 15) / 16;
        if (!distinct(t)) return;
        // butterfly passes
        std::fill(live.begin(), live.end(), 0);
        lv.clear();
        uint32_t W = 0;
        for (uint32_t k = 0; k < npp; ++k) {
            W |= st(t - 1, k);
            live[st(t - 1, k)] = 1;
            lv.push_back(st(t - 1, k));
        }
        // D: the hidden states below some state of year t - 1 (U's
        // support); N: those below some state of year t (U's reads, the
        // union of the year's K lists); M(rem): the positions whose value
        // still reaches N by the butterflies over the patches rem (N's
        // up-closure over rem) -- a pass reads live positions in M(before)
        // and writes positions in M(after) only
        std::vector<uint8_t> Dm(ncube, 0), Nm(ncube, 0), Mb(ncube), Ma(ncube);
        for (uint32_t k = 0; k < npp; ++k) Dm[st(t - 1, k)] = 1;
        for (uint32_t bit = 1; bit < ncube; bit <<= 1)
            for (uint32_t q = 0; q < ncube; ++q)
                if ((q & bit) && Dm[q]) Dm[q ^ bit] = 1;
        uint32_t nused = 0;  // patches set in some j of N
        for (uint32_t l = 0; l < npc; ++l) {
            const uint32_t key = st(t, l) & W;
            for (uint32_t j = key;; j = (j - 1) & key) {
                if (Dm[j] && !Nm[j]) {
                    Nm[j] = 1;
                    nused |= j;
                }
                if (!j) break;
            }
        }
        auto upclose = [&](uint32_t rem, std::vector<uint8_t> &M) {
            M = Nm;
            for (uint32_t bit = 1; bit < ncube; bit <<= 1)
                if (rem & bit)
                    for (uint32_t q = 0; q < ncube; ++q)
                        if (!(q & bit) && M[q]) M[q | bit] = 1;
        };
        // the patches of W: first those set in no j of N (each halves what
        // later passes touch), then greedily the one adding the fewest new
        // positions (ties: fewest values to move)
        std::vector<uint32_t> border;
        {
            std::vector<uint8_t> lt(live);
            std::vector<uint32_t> l2(lv);
            for (int phase = 0; phase < 2; ++phase)
                for (uint32_t rem = W & (phase ? nused : ~nused); rem;) {
                    uint32_t best = 0, bnew = ~0u, bpairs = ~0u;
                    for (uint32_t rr = rem; rr; rr &= rr - 1) {
                        const uint32_t bit = rr & (0u - rr);
                        uint32_t nw = 0, pr = 0;
                        for (uint32_t a : l2)
                            if (a & bit) {
                                ++pr;
                                nw += !lt[a ^ bit];
                            }
                        if (nw < bnew || (nw == bnew && pr < bpairs)) {
                            best = bit;
                            bnew = nw;
                            bpairs = pr;
                        }
                    }
                    rem &= ~best;
                    border.push_back((uint32_t)__builtin_ctz(best));
                    const size_t n2 = l2.size();
                    for (size_t i = 0; i < n2; ++i)
                        if ((l2[i] & best) && !lt[l2[i] ^ best]) {
                            lt[l2[i] ^ best] = 1;
                            l2.push_back(l2[i] ^ best);
                        }
                }
        }
        eng->hs_pbase[t] = (uint32_t)eng->hs_pass.size();
        const size_t npass = (border.size() + radix - 1) / radix;
        uint32_t remw = W;
        for (size_t ip = 0, b0 = 0; ip < npass; ++ip) {
            // passes of near-equal size (radix 4: 10 patches 4 + 3 + 3)
            const uint32_t r = (uint32_t)((border.size() - b0 + (npass - ip) - 1) / (npass - ip));
            uint32_t bp[kHsRadix] = {}, mask = 0, bits = 0;
            for (uint32_t k = 0; k < r; ++k) {
                bp[k] = border[b0 + k];
                mask |= 1u << bp[k];
                bits |= bp[k] << (5 * k);
            }
            b0 += r;
            upclose(remw, Mb);
            remw &= ~mask;
            upclose(remw, Ma);
            auto dep = [&](uint32_t q) {
                uint32_t o = 0;
                for (uint32_t k = 0; k < r; ++k)
                    if (q & (1u << k)) o |= 1u << bp[k];
                return o;
            };
            std::map<uint32_t, uint32_t> cos;  // g -> mask of positions read
            for (uint32_t a : lv) {
                if (!Mb[a]) continue;
                uint32_t q = 0;
                for (uint32_t k = 0; k < r; ++k)
                    if (a & (1u << bp[k])) q |= 1u << k;
                cos[a & ~mask] |= 1u << q;
            }
            const uint32_t base = (uint32_t)eng->hs_ppos.size();
            std::map<uint32_t, std::vector<uint32_t>> bymask;  // read | write << 16 -> its cosets
            for (auto &kv : cos) {
                uint32_t cl = kv.second;  // the read positions' subsets
                cl |= (cl & 0xaaaau) >> 1;
                cl |= (cl & 0xccccu) >> 2;
                cl |= (cl & 0xf0f0u) >> 4;
                cl |= (cl & 0xff00u) >> 8;
                uint32_t outm = 0;
                for (uint32_t q = 0; q < (1u << r); ++q)
                    if (((cl >> q) & 1u) && Ma[kv.first | dep(q)]) outm |= 1u << q;
                bymask[kv.second | outm << 16].push_back(kv.first);
            }
            // cosets grouped by masks, pts / 64 ... a wave's worth at a time
            // (64 / pts cosets a wave), each wave padded with copies of its
            // first coset (a lane of the same wave: identical values)
            const uint32_t cpw = 64u / pts;
            for (auto &mv : bymask)
                for (size_t i = 0; i < mv.second.size(); i += cpw)
                    for (uint32_t k = 0; k < cpw; ++k)
                        eng->hs_ppos.push_back(make_uint2(i + k < mv.second.size() ? mv.second[i + k] : mv.second[i],
                                                          mv.first));
            for (auto &kv : cos) {
                uint32_t cl = kv.second;
                cl |= (cl & 0xaaaau) >> 1;
                cl |= (cl & 0xccccu) >> 2;
                cl |= (cl & 0xf0f0u) >> 4;
                cl |= (cl & 0xff00u) >> 8;
                uint32_t outm = 0;
                for (uint32_t q = 0; q < (1u << r); ++q)
                    if (((cl >> q) & 1u) && Ma[kv.first | dep(q)]) outm |= 1u << q;
                fb += 2.0 * (double)r * (double)(1u << (r - 1)) + (ip + 1 == npass ? (double)(1u << r) : 0.0);
                for (uint32_t q = 0; q < (1u << r); ++q)
                    if (((outm >> q) & 1u) && !live[kv.first | dep(q)]) {
                        live[kv.first | dep(q)] = 1;
                        lv.push_back(kv.first | dep(q));
                    }
            }
            eng->hs_pass.push_back(make_uint4(bits, r, (uint32_t)eng->hs_ppos.size() - base, base));
        }
        // the year's states in tile order
        std::vector<uint32_t> ord(npc);
        for (uint32_t l = 0; l < npc; ++l) ord[l] = l;
        std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) {
            const uint32_t bx = st(t, x), by = st(t, y);
            return (bx & W) != (by & W) ? (bx & W) < (by & W) : bx < by;
        });
        eng->hs_dbase[t] = (uint32_t)eng->hs_dpos.size();
        for (uint32_t i = 0; i < ncol * 16; ++i) eng->hs_dpos.push_back(i < npc ? st(t, ord[i]) : ~0u);
        std::vector<uint32_t> nch(ncol);
        std::vector<uint32_t> K;
        for (uint32_t tile = 0; tile < ncol; ++tile) {
            K.clear();
            for (uint32_t i = 16 * tile; i < std::min(16 * tile + 16, npc); ++i) {
                const uint32_t key = st(t, ord[i]) & W;
                for (uint32_t j = key;; j = (j - 1) & key) {  // subsets of key (with j = 0 last)
                    if (Dm[j]) K.push_back(j);
                    if (!j) break;
                }
            }
            std::sort(K.begin(), K.end());
            K.erase(std::unique(K.begin(), K.end()), K.end());
            const size_t start = eng->hs_kt.size();
            for (uint32_t j : K) {
                eng->hs_kt.push_back(j * pts * 8u);
                for (uint32_t i = 16 * tile; i < 16 * tile + 16; ++i) {
                    uint32_t o = zero;
                    if (i < npc && !(j & ~st(t, ord[i]))) {
                        auto it = item.find(((uint64_t)j << 32) | st(t, ord[i]));
                        if (it == item.end()) return;
                        o = it->second;
                    }
                    eng->hs_cidx.push_back(o * 8u);
                }
            }
            while ((eng->hs_kt.size() - start) % cw) {
                eng->hs_kt.push_back(0u);
                for (uint32_t l = 0; l < 16; ++l) eng->hs_cidx.push_back(zero * 8u);
            }
            nch[tile] = (uint32_t)((eng->hs_kt.size() - start) / cw);
            ktile[tile] = make_uint2((uint32_t)start, nch[tile]);
            fm += 2.0 * 16.0 * (double)(eng->hs_kt.size() - start);
        }
        // free park blocks
        std::vector<uint8_t> used(ncube / 16, 0);
        for (uint32_t l = 0; l < npc; ++l) used[st(t, l) / 16] = 1;
        uint32_t room = 0;
        for (uint32_t b = 0; b < ncube / 16 && room < 16; ++b)
            if (!used[b]) eng->hs_pk[(size_t)t * 16 + room++] = b * 16;
        plan_waves(nch, tmaxit, 1u, room, wtmp.data(), nw);
        for (uint32_t i = 0; i < nw * tmaxit; ++i) {
            const uint2 kt2 = ktile[wtmp[i].y & 0xffu];
            eng->hs_wplan[(size_t)t * nw * tmaxit + i] =
                (wtmp[i].y >> 24) ? make_uint4(wtmp[i].x, wtmp[i].y, kt2.x, kt2.y) : make_uint4(wtmp[i].x, wtmp[i].y, 0u, 1u);
        }
    }
    eng->hs_pbase[eng->tmax] = (uint32_t)eng->hs_pass.size();
    // the store positions per (16 positions of dpos, lane group kk): entries
    // kk + 4 r, r = 0 .. 3, 16 bits each (0xffff: padding)
    eng->hs_dpk.assign(eng->hs_dpos.size() / 16 * 4, make_uint2(0u, 0u));
    for (size_t b = 0; b < eng->hs_dpos.size() / 16; ++b)
        for (uint32_t kq = 0; kq < 4; ++kq) {
            uint32_t w[4];
            for (uint32_t r = 0; r < 4; ++r) {
                const uint32_t ps = eng->hs_dpos[b * 16 + kq + 4 * r];
                w[r] = ps == ~0u ? 0xffffu : ps;
            }
            eng->hs_dpk[b * 4 + kq] = make_uint2(w[0] | w[1] << 16, w[2] | w[3] << 16);
        }
    if (eng->hs_kt.empty()) eng->hs_kt.push_back(0u);
    if (eng->hs_ppos.empty()) eng->hs_ppos.push_back(make_uint2(0u, 0u));
    if (eng->hs_pass.empty()) eng->hs_pass.push_back(make_uint4(0u, 0u, 0u, 0u));
    eng->hs_mfma_pt = fm;
    eng->hs_flops_pt = fb + fm + (double)eng->np[eng->tmax - 1];
    eng->hs_rt = rt;
    eng->hs_nb = nb;
    eng->hs_nw = nw;
    if (const char *pv = eng->opts.get("MDP_HS_PROBE")) eng->hs_probe = (uint32_t)atoi(pv) & 7u;
    eng->hs = hs_lds(eng) <= device_lds_max() && eng->hs_kt.size() < (1u << 26);
}

int build_wide_plan(mdp_engine *eng, const mdp_problem *p)
{
    int rc = build_direct_plan(eng, p);
    if (rc) return rc;
    // Q rows with at least one zero slot past the coefficients (slot ncoef:
    // k_fwd_mma's gathers of absent coefficients read it)
    eng->ldQ = ((size_t)eng->ncoef_d + 2) & ~(size_t)1;
    double f = 2.0 * (eng->maxA + 1) + 2.0 * eng->np[eng->tmax - 1];
    for (uint32_t d : eng->udesc_d) f += 3.0 * (((d >> kOffBits) & 31u) + 1.0) + 2.0;
    eng->wide_flops_pt = f;
    // k_fwd_mma's tables (c-independent): years of at most 256 states; per
    // year its K entries (k, |A_k|, m), padded to whole pipeline chunks with
    // entries naming the descriptor row npp (every transition absent), and the
    // transition descriptors [k][2^sh >= npcp] (Q-row offset | nX << kOffBits;
    // an absent transition names the zero slot with nX = 0)
    // MDP_WIDE_MMA: 0 -> k_fwd_wide; 1 -> round 5's k_fwd_mma (<= 256
    // states); 2 -> k_fwd_mmt (<= 1 024 states); 3 -> k_fwd_hs (nvar <= 10;
    // else k_fwd_mmt); unset -> k_fwd_hs for years of more than 64 states,
    // else k_fwd_mmt (measured, profiles/r06/hs: k_fwd_hs 1.3x / 4.4x / 5.2x
    // / 5.8x faster on 128 / 256 / 512 / 1 024 states, 1.27x slower on 64)
    const char *mv = eng->opts.get("MDP_WIDE_MMA");
    const int mmode = mv ? atoi(mv) : (eng->npmax > 64 ? 3 : 2);
    eng->mmt = false;
    eng->hs = false;
    if (mmode == 3) build_hs_plan(eng);
    if (mmode == 2 || (mmode == 3 && !eng->hs)) build_mmt_plan(eng);
    eng->mma = false;
    if (eng->npmax <= 256 && eng->maxA <= 24) {
        if (mmode == 1) {
            const uint32_t npm = eng->npmax <= 64 ? 64u : eng->npmax <= 128 ? 128u : 256u;
            const uint32_t pts = mma_pts(npm), ps = mma_ps(npm);
            const uint32_t none = (uint32_t)eng->ncoef_d;  // the zero slot, nX = 0
            eng->mma_npm = npm;
            eng->mma_kt.clear();
            eng->mma_desc.clear();
            eng->mma_kbase.assign(eng->tmax + 1, 0u);
            eng->mma_dbase.assign(eng->tmax + 1, 0u);
            eng->mma_ktmax = 16;
            size_t ub = 0;
            bool pad_overflow = false;
            for (uint32_t t = 1; t < eng->tmax; ++t) {
                const uint32_t npp = eng->np[t - 1], npc = eng->np[t], npcp = (npc + 15) / 16 * 16;
                uint32_t ld = 16;
                while (ld < npcp) ld *= 2;
                eng->mma_kbase[t] = (uint32_t)eng->mma_kt.size();
                eng->mma_dbase[t] = (uint32_t)eng->mma_desc.size();
                for (uint32_t k = 0; k < npp; ++k) {
                    const uint32_t a = eng->udesc_d[ub + k] >> 27;  // |A_k| (any use from k; l = 0)
                    for (uint32_t m = 0; m <= a; ++m)  // Va row k, xp row a - m, yp row m (bytes); m; k
                        eng->mma_kt.push_back(make_uint2((k * pts * 8u) | (((a - m) * ps * 8u) << 16),
                                                         (m * ps * 8u) | (m << 16) | (k * kMmaDummy)));
                }
                // padding names descriptor row npp through the 8-bit k field:
                // row 256 would wrap to row 0 (the advisor's round-5 finding),
                // so a 256-state year that needs padding leaves k_fwd_mma
                if (eng->mma_kt.size() % (4 * kMmaU) && npp > 255) pad_overflow = true;
                while (eng->mma_kt.size() % (4 * kMmaU)) eng->mma_kt.push_back(make_uint2(0u, npp * kMmaDummy));
                eng->mma_ktmax = std::max<uint32_t>(eng->mma_ktmax, (uint32_t)eng->mma_kt.size() - eng->mma_kbase[t]);
                for (uint32_t k = 0; k <= npp; ++k)
                    for (uint32_t l = 0; l < ld; ++l) {
                        uint32_t dv = none;
                        if (k < npp && l < npc) {
                            const uint32_t dsc = eng->udesc_d[ub + (size_t)l * npp + k];
                            dv = (dsc & kOffMask) | (((dsc >> kOffBits) & 31u) << kOffBits);
                        }
                        eng->mma_desc.push_back(dv);
                    }
                ub += (size_t)npp * npc;
            }
            eng->mma_kbase[eng->tmax] = (uint32_t)eng->mma_kt.size();
            eng->mma_dbase[eng->tmax] = (uint32_t)eng->mma_desc.size();
            // per year and wave its work item (k_fwd_mma): column tile, K
            // slice of S (at most 16 waves; slice 1 in the destination rows,
            // later ones in the rows past the year's column tiles; at least
            // two chunks each), chunk range
            eng->mma_wplan.assign((size_t)(eng->tmax + 1) * 16, make_uint2(0u, 0u));
            for (uint32_t t = 1; t < eng->tmax; ++t) {
                const uint32_t ncol = (eng->np[t] + 15) / 16, npcp = ncol * 16;
                const uint32_t nch = (eng->mma_kbase[t + 1] - eng->mma_kbase[t]) / (4 * kMmaU);
                const uint32_t room = 2 + (mma_rows(npm) - npcp) / npcp;
                const uint32_t S = std::min(std::min(16 / ncol, room), std::max(1u, nch / 2));
                for (uint32_t wv = 0; wv < 16; ++wv) {
                    const uint32_t item = wv % ncol, ks = wv / ncol;
                    const uint32_t cb = nch * ks / S, ce = nch * (ks + 1) / S;
                    eng->mma_wplan[(size_t)t * 16 + wv] =
                        make_uint2(cb | ce << 16, item | ks << 8 | S << 16 | (wv < ncol * S ? 1u : 0u) << 24);
                }
            }
            // (chunk reads past a year's entries are clamped into it; one
            // chunk of slack keeps the last year's clamp in the table)
            for (uint32_t i = 0; i < 4 * kMmaU; ++i) eng->mma_kt.push_back(make_uint2(0u, 0u));
            if (eng->mma_desc.empty()) eng->mma_desc.push_back(none);
            const size_t lmax = device_lds_max();
            eng->mma = mma_lds(eng) <= lmax && none <= kOffMask && !pad_overflow;
        }
    }
    return MDP_OK;
}


constexpr size_t kQrowsLdsMax = 160 * 1024;
constexpr size_t kFusedLdsMax = 64 * 1024;  // fused forward kernel: every table of one column

// k_qrows LDS for cb c values per workgroup: Z, var-column S, Pc, Q CSR
size_t qrows_lds(const mdp_engine *eng, uint32_t cb)
{
    const size_t nv = eng->nvar <= 8 ? 8 : eng->nvar <= 16 ? 16 : 24;  // k_qrows NV
    return ((((size_t)cb * eng->nj + 1) & ~(size_t)1) + (size_t)eng->nj * (cb * nv + 2) + (size_t)cb * eng->npl_slots) *
               sizeof(double) +
           ((size_t)eng->ncoef_d + 1 + eng->qitem.size()) * sizeof(uint32_t);  // (items stay in registers)
}

// Z rows for a grid whose |c| <= cmax.  Z_j(c) = prod over the always-zero
// columns k of max(0, 1 - c S[j][k]) splits by the size of |c| S:
//  * |c| S <= 2^-55: the factor is exactly 1.0 -- dropped;
//  * 2^-55 < |c| S <= kZTau ("small"): never clamped, and their product is
//    exp(sum log(1 - c S)) = exp(-sum_i c^i P_i / i) with the power sums
//    P_i = sum_small S^i.  The series stops after kZTerms terms: the rest is
//    below sum_small (c S)^(kZTerms+1) / (kZTerms+1) <= 256 * 2^-63 / 9
//    < 2^-58 relative per 256 small columns (exp: ~1 ulp), so Z keeps
//    double precision while a row costs kZTerms FMAs and one exp instead of
//    an FMA and a multiply per column (config 3: 248 -> <= 24 columns a row);
//  * the rest ("large", |c| S > kZTau or not finite) stay explicit factors,
//    the largest first (the clamp test reads it).
// zs[k][row] / zsT[row][k] hold the large columns (kmax = the longest row
// rounded up to 8, zero padding = factor 1.0); zc[row][kZTerms] the series
// coefficients P_i / i (zero for a row without small columns: exp(0) = 1).
constexpr double kZTau = 0x1p-7;
constexpr int kZTerms = kZTermsDev;

void z_split(const mdp_engine *eng, uint32_t js, double cmax, std::vector<double> &large, double *coef,
             std::vector<uint32_t> *cols = nullptr)
{
    const uint32_t n = eng->n;
    large.clear();
    if (cols) cols->clear();
    size_t imax = 0;
    double pw[kZTerms] = {};
    for (uint32_t k = 0; k < n; ++k) {
        if (eng->isvar[k]) continue;
        const double sv = eng->Sj[(size_t)js * n + k];
        const double x = cmax * sv;
        if (x <= 0x1p-55) continue;  // false for NaN / inf: kept
        if (x <= kZTau) {
            double t = sv;
            for (int i = 0; i < kZTerms; ++i, t *= sv) pw[i] += t;
            continue;
        }
        if (!large.empty() && sv > large[imax]) imax = large.size();
        large.push_back(sv);
        if (cols) cols->push_back(k);
    }
    if (!large.empty()) std::swap(large[0], large[imax]);
    if (cols && !cols->empty()) std::swap((*cols)[0], (*cols)[imax]);
    if (coef)
        for (int i = 0; i < kZTerms; ++i) coef[i] = pw[i] / (double)(i + 1);
}

int upload_qrows_tables(const mdp_engine *eng, DevCtx &d, double cmax)
{
    const uint32_t n = eng->n, nj = eng->nj;
    (void)n;
    std::vector<std::vector<double>> rows(nj);
    std::vector<double> zc((size_t)nj * kZTerms + 1, 0.0);
    size_t kmax = 0;
    for (uint32_t js = 0; js < nj; ++js) {
        z_split(eng, js, cmax, rows[js], &zc[(size_t)js * kZTerms]);
        kmax = std::max(kmax, rows[js].size());
    }
    kmax = (kmax + 7) & ~(size_t)7;
    std::vector<double> zs(kmax * nj + 1, 0.0);  // [k][row]: the fused kernel's image
    for (uint32_t js = 0; js < nj; ++js)
        for (size_t k = 0; k < rows[js].size(); ++k) zs[k * nj + js] = rows[js][k];
    std::vector<double> zsT(kmax * nj + 1, 0.0);  // [row][k]: k_zrows (device copy)
    for (uint32_t js = 0; js < nj; ++js)
        for (size_t k = 0; k < rows[js].size(); ++k) zsT[js * kmax + k] = rows[js][k];
    int rc;
    if ((rc = dev_reserve(&d.zs, &d.cap_zs, zsT.size()))) return rc;
    HIP_TRY(hipMemcpy(d.zs, zsT.data(), zsT.size() * sizeof(double), hipMemcpyHostToDevice));
    // k_qrows' copy: row js's product chain q (columns k = q mod 4) contiguous
    std::vector<double> zsq(kmax * nj + 2, 0.0);  // + a double2 k_qrows may read at kmax 0
    for (uint32_t js = 0; js < nj; ++js)
        for (size_t k = 0; k < kmax; ++k) zsq[js * kmax + (k % 4) * (kmax / 4) + k / 4] = zsT[js * kmax + k];
    if ((rc = dev_reserve(&d.zsq, &d.cap_zsq, zsq.size()))) return rc;
    HIP_TRY(hipMemcpy(d.zsq, zsq.data(), zsq.size() * sizeof(double), hipMemcpyHostToDevice));
    if ((rc = dev_reserve(&d.zc, &d.cap_zc, zc.size()))) return rc;
    HIP_TRY(hipMemcpy(d.zc, zc.data(), zc.size() * sizeof(double), hipMemcpyHostToDevice));
    d.zs_cmax = cmax;
    d.zs_len = (uint32_t)(kmax * nj);
    d.zs_kmax = (uint32_t)kmax;
    // no fused kernel on the wide path, for a chunked series or Q rows built in HBM
    if (eng->wide || eng->qglobal || !eng->chunks.empty() || eng->jit_plan.vlds) return MDP_OK;
    // the fused kernel's column tables: one contiguous image it copies to LDS
    // (with zpad, all KZ zs rows, zero past kmax: the kernel reads them unmasked)
    const MdpJitPlan &pl = eng->jit_plan;
    const size_t kimg = pl.zpad ? std::max<size_t>(kmax, std::max<uint32_t>(8u, pl.kzmax)) : kmax;
    const size_t ct = ((size_t)pl.off_zs + kimg * nj + 127) & ~(size_t)127;
    std::vector<double> img(ct, 0.0);
    for (uint32_t js = 0; js < nj; ++js)  // (the columns of j marked +inf: pressure fmin(c inf, 1) = 1.0)
        for (uint32_t b = 0; b < eng->nvar; ++b)
            img[(size_t)js * eng->nvar + b] = ((eng->cj_bits[js] >> (eng->nvar - 1 - b)) & 1u)
                                                   ? HUGE_VAL
                                                   : eng->Sj[(size_t)js * n + eng->var_cols[b]];
    uint2 *it = (uint2 *)(img.data() + pl.off_it);
    for (uint32_t i = 0; i < eng->nitems; ++i) {
        const uint32_t r = eng->itemRow[i];
        it[i] = make_uint2(eng->itemB[i] | ((r & 0xffu) << 24), eng->cj_bits[r] | ((r >> 8) << 24));
    }
    memcpy(img.data() + pl.off_qs, eng->qstart.data(), eng->qstart.size() * sizeof(uint32_t));
    memcpy(img.data() + pl.off_zc, zc.data(), (size_t)nj * kZTerms * sizeof(double));
    if (!eng->qitem.empty())
        memcpy(img.data() + pl.off_qi, eng->qitem.data(), eng->qitem.size() * sizeof(uint32_t));
    {
        const std::vector<uint32_t> rq = mdp_jit_reversed_index(pl.udesc, pl.ldQ);
        memcpy(img.data() + pl.off_rq, rq.data(), rq.size() * sizeof(uint32_t));
    }
    for (size_t k = 0; k < kmax; ++k)  // zs pairs (k, k+1) of a row adjacent: one ds_read_b128
        for (uint32_t js = 0; js < nj; ++js) img[pl.off_zs + ((k / 2) * nj + js) * 2 + (k & 1)] = zs[k * nj + js];
    if ((rc = dev_reserve(&d.coltab, &d.cap_coltab, ct))) return rc;
    HIP_TRY(hipMemcpy(d.coltab, img.data(), ct * sizeof(double), hipMemcpyHostToDevice));
    d.ct_len = (uint32_t)ct;
    return MDP_OK;
}

// Compile (hipRTC, cached) the engine's forward kernel: variant 0 reading,
// 1 fused, 2 reading at kJitKblockTall threads (a column of a tall grid in
// half the blocks: its Q row staged half as often).
constexpr int kJitKblockTall = 512;
int jit_build(mdp_engine *eng, int variant)
{
    const bool fused = variant == 1;
    if (!eng->jit_code[variant].empty()) return MDP_OK;
    MdpJitPlan plan = eng->jit_plan;
    plan.fused = fused;
    if (variant == 2) {  // the reading kernel's points per lane, more threads
        plan.epl = eng->jit_epl > 0 ? eng->jit_epl : mdp_jit_default_epl(plan.udesc);
        plan.kblock = kJitKblockTall;
        const std::string src = mdp_jit_forward_source(plan);
        if (mdp_jit_compile(src, eng->jit_code[2], eng->jit_log) != 0)
            return mdp_set_error(MDP_EHIP, "hipRTC compilation of the forward kernel failed: %s", eng->jit_log.c_str());
        eng->jit_src[2] = src;
        return MDP_OK;
    }
    // the reading variant's shape (e rows per block = kblock x epl, which
    // set_grid_dev's block count uses before it picks the variant)
    const int epl_r = plan.epl > 0 ? plan.epl : mdp_jit_default_epl(plan.udesc);
    const int kb_r = plan.kblock > 0 ? plan.kblock : kBlock;
    eng->jit_epl = epl_r;
    eng->jit_kblock = (uint32_t)kb_r;
    if (fused && !eng->jit_shape_env) {
        // the same e rows per block as the reading variant (kb_r x epl_r, the
        // grid shape is shared), the forward at its points per lane, and
        // twice the threads for the column-table prologue (pro 2): a
        // forward at one point per lane was LDS-bound (each broadcast pair
        // read feeds half the FMAs), while the prologue wants every thread
        plan.kblock = kb_r;
        plan.epl = epl_r;
        plan.pro = 2;
    }
    if (fused) {  // at most 1 024 threads a workgroup: fewer prologue threads, then fewer columns
        const int fc = std::max(1, plan.fused_cols);
        if (plan.kblock * fc * std::max(1, plan.pro) > 1024) plan.pro = 1;
        if (plan.kblock * fc > 1024) plan.fused_cols = std::max(1, 1024 / std::max(1, plan.kblock));
        eng->jit_plan.fused_cols = plan.fused_cols;  // the launch's columns per workgroup
    }
    const std::string src = mdp_jit_forward_source(plan);
    if (fused) {
        eng->jit_epl_fused = plan.epl;
        eng->jit_kblock_fused = (uint32_t)plan.kblock;
        eng->jit_pro_fused = (uint32_t)std::max(1, plan.pro);
    }
    eng->jit_flops_pt = plan.flops_pt;
    if (const char *dump = eng->opts.get("MDP_JIT_DUMP")) {  // <path>.hip (reading) / <path>.fused.hip
        if (FILE *f = fopen((std::string(dump) + (fused ? ".fused.hip" : ".hip")).c_str(), "w")) {
            fputs(src.c_str(), f);
            fclose(f);
        }
    }
    if (mdp_jit_compile(src, eng->jit_code[variant], eng->jit_log) != 0)
        return mdp_set_error(MDP_EHIP, "hipRTC compilation of the forward kernel failed: %s",
                             eng->jit_log.c_str());
    eng->jit_src[variant] = src;
    return MDP_OK;
}

// Compile every chunk kernel of a long series (threads: hipRTC programs are
// independent).
int jit_build_chunks(mdp_engine *eng)
{
    const size_t nch = eng->chunks.size();
    if (eng->chunk_code.size() == nch) return MDP_OK;
    std::vector<std::vector<char>> code(nch);
    std::vector<std::string> logs(nch);
    std::vector<int> rcs(nch, 0);
    std::vector<std::string> srcs(nch);
    double flops = 0.0;
    for (size_t i = 0; i < nch; ++i) {
        srcs[i] = mdp_jit_forward_source(eng->chunks[i]);
        flops += eng->chunks[i].flops_pt;
        if (const char *dump = eng->opts.get("MDP_JIT_DUMP"))
            if (FILE *f = fopen((std::string(dump) + ".chunk" + std::to_string(i) + ".hip").c_str(), "w")) {
                fputs(srcs[i].c_str(), f);
                fclose(f);
            }
    }
    {
        std::vector<std::thread> th;
        size_t nt = std::min<size_t>(8, nch);
        if (const char *tv = eng->opts.get("MDP_JIT_THREADS")) nt = std::max<size_t>(1, std::min<size_t>(nch, atoi(tv)));
        const bool verbose = eng->opts.get("MDP_JIT_VERBOSE") != nullptr;
        for (size_t t = 0; t < nt; ++t)
            th.emplace_back([&, t]() {
                for (size_t i = t; i < nch; i += nt) {
                    const auto t0 = std::chrono::steady_clock::now();
                    rcs[i] = mdp_jit_compile(srcs[i], code[i], logs[i]);
                    if (verbose)
                        fprintf(stderr, "chunk %zu: %zu uses, %.2f s\n", i, eng->chunks[i].udesc.size(),
                                std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
                }
            });
        for (auto &x : th) x.join();
    }
    for (size_t i = 0; i < nch; ++i)
        if (rcs[i]) {
            eng->jit_log = logs[i];
            return mdp_set_error(MDP_EHIP, "hipRTC compilation of forward chunk %zu failed: %s", i, logs[i].c_str());
        }
    eng->chunk_code = std::move(code);
    eng->chunk_src = std::move(srcs);
    eng->jit_epl = eng->chunks[0].epl;
    eng->jit_kblock = (uint32_t)eng->chunks[0].kblock;
    eng->jit_flops_pt = flops;
    return MDP_OK;
}

// Load a code object; if the runtime refuses it (a stale or foreign object
// from the disk cache), rebuild it from its source once and retry.
hipError_t load_module(std::vector<char> &code, const std::string &src, hipModule_t *m)
{
    hipError_t e = hipModuleLoadData(m, code.data());
    if (e == hipSuccess || src.empty()) return e;
    std::string log;
    if (mdp_jit_compile(src, code, log, true) != 0) return e;
    return hipModuleLoadData(m, code.data());
}

// Load a forward kernel variant (jit_build's) into the device, compiling it if needed.
int jit_load(mdp_engine *eng, DevCtx &d, int variant)
{
    if (!eng->chunks.empty()) {  // a long series: its chunk kernels (never fused)
        const size_t nch = eng->chunks.size();
        if (d.cfn.size() == nch) return MDP_OK;
        int rc = jit_build_chunks(eng);
        if (rc) return rc;
        HIP_TRY(hipSetDevice(d.device));
        // every chunk loads into locals first and is committed to the device
        // context only when all have: a failure part-way leaves nothing
        // loaded, so a later call retries instead of running some chunks
        std::vector<hipModule_t> mods;
        std::vector<hipFunction_t> fns;
        std::vector<uint32_t *> qidx;
        auto unload = [&]() {
            for (hipModule_t m : mods) (void)hipModuleUnload(m);
            for (uint32_t *q : qidx)
                if (q) (void)hipFree(q);
        };
        for (size_t i = 0; i < nch; ++i) {
            hipModule_t m;
            hipFunction_t f;
            hipError_t e = load_module(eng->chunk_code[i], i < eng->chunk_src.size() ? eng->chunk_src[i] : std::string(), &m);
            if (e == hipSuccess) {
                mods.push_back(m);
                e = hipModuleGetFunction(&f, m, "mdp_fwd_jit");
            }
            if (e != hipSuccess) {
                unload();
                return mdp_set_error(MDP_EHIP, "loading forward chunk %zu failed: %s", i, hipGetErrorString(e));
            }
            fns.push_back(f);
            uint32_t *qi = nullptr;
            if (!eng->chunks[i].qidx.empty() && (rc = dev_upload(&qi, eng->chunks[i].qidx))) {
                unload();
                return rc;
            }
            qidx.push_back(qi);
        }
        d.cmod = std::move(mods);
        d.cfn = std::move(fns);
        d.cqidx = std::move(qidx);
        return MDP_OK;
    }
    if (d.jit_fn[variant]) return MDP_OK;
    int rc = jit_build(eng, variant);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(d.device));
    hipModule_t m = nullptr;
    hipFunction_t f = nullptr;
    HIP_TRY(load_module(eng->jit_code[variant], eng->jit_src[variant], &m));
    const hipError_t e = hipModuleGetFunction(&f, m, "mdp_fwd_jit");
    if (e != hipSuccess) {
        (void)hipModuleUnload(m);
        return mdp_set_error(MDP_EHIP, "hipModuleGetFunction(mdp_fwd_jit) failed: %s", hipGetErrorString(e));
    }
    d.jit_mod[variant] = m;
    d.jit_fn[variant] = f;
    return MDP_OK;
}

// The fused forward kernel keeps its column's tables (ct_len doubles,
// dynamic LDS), Z, Pc and Q in LDS.
size_t fused_lds(const mdp_engine *eng, size_t ct_len)
{
    const size_t fc = (size_t)eng->jit_plan.fused_cols;
    return (ct_len + 2 + fc * (eng->nj + eng->nitems + 2 * eng->ldQ)) * sizeof(double);  // + staging scratch
}

constexpr size_t kWidePgBytes = 256ull << 20;  // wide path: item-factor chunk
constexpr size_t kHsPgBytes = 2048ull << 20;   // k_fwd_hs: item factors of the columns of one launch
constexpr size_t kWideVBytes = 1ull << 30;     // wide path: state-vector scratch

// k_fwd_wide: per-lane x^r, y^r tables, r <= maxA
size_t wide_lds(const mdp_engine *eng) { return 2 * ((size_t)eng->maxA + 1) * kBlock * sizeof(double); }

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

// The generic path's device tables: colonisation sums S of every state
// (k_colsum), the binomial table, the pair plans, k_coefs' LDS limit.
int init_generic(mdp_engine *eng, DevCtx &d, const mdp_problem *p)
{
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
        (rc = dev_upload(&d.pairOff, eng->pairOff)) || (rc = dev_upload(&d.udesc, eng->udesc)) ||
        (rc = dev_upload(&d.pairPart0, eng->pairPart0)) || (rc = dev_upload(&d.partP, eng->partP)) ||
        (rc = dev_upload(&d.partK0, eng->partK0)) ||
        (rc = dev_upload(&d.prog, eng->prog)) ||
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
        const void *fns[] = {
            (const void *)k_coefs<true, true, 8>,   (const void *)k_coefs<true, true, 16>,
            (const void *)k_coefs<true, true, 24>,  (const void *)k_coefs<false, true, 8>,
            (const void *)k_coefs<false, true, 16>, (const void *)k_coefs<false, true, 24>,
            (const void *)k_coefs<false, false, 8>, (const void *)k_coefs<false, false, 16>,
            (const void *)k_coefs<false, false, 24>};
        for (const void *fn : fns)
            HIP_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)eng->coef_lds));
    }
    return MDP_OK;
}

int init_device(mdp_engine *eng, DevCtx &d, const mdp_problem *p)
{
    HIP_TRY(hipSetDevice(d.device));
    HIP_TRY(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
    int rc = MDP_OK;
    // the generic path's tables (k_zpv / k_coefs / k_forward: colonisation
    // sums of every state, binomials, pair plans) only for an engine that
    // runs it: the direct and wide paths never touch them, so their set-up
    // does not load the library's precompiled kernels at all (CLI start-up)
    if (!eng->jit && !eng->wide && (rc = init_generic(eng, d, p))) return rc;
    if (eng->jit || eng->wide) {
        std::vector<double> sv((size_t)eng->nj * eng->nvar + 1, 0.0);
        for (uint32_t js = 0; js < eng->nj; ++js)
            for (uint32_t b = 0; b < eng->nvar; ++b)
                sv[(size_t)js * eng->nvar + b] = ((eng->cj_bits[js] >> (eng->nvar - 1 - b)) & 1u)
                                                      ? HUGE_VAL  // column of j: pC = fmin(c inf, 1) = 1.0
                                                      : eng->Sj[(size_t)js * eng->n + eng->var_cols[b]];
        std::vector<uint2> items(eng->nitems + 1, make_uint2(0u, 0u));
        for (uint32_t i = 0; i < eng->nitems; ++i) {
            const uint32_t r = eng->itemRow[i];
            items[i] = make_uint2(eng->itemB[i] | ((r & 0xffu) << 24), eng->cj_bits[r] | ((r >> 8) << 24));
        }
        std::vector<uint32_t> qitem = eng->qitem;
        qitem.push_back(0u);
        if ((rc = dev_upload(&d.sv, sv)) || (rc = dev_upload(&d.items, items)) ||
            (rc = dev_upload(&d.qstart, eng->qstart)) || (rc = dev_upload(&d.qitem, qitem)) ||
            (rc = dev_upload(&d.qslot, eng->qslot)) || (rc = dev_upload(&d.qlane, eng->qlane)) ||
            (rc = dev_upload(&d.islot, eng->islot)))
            return rc;
        if (eng->wide) {
            if ((rc = dev_upload(&d.np_d, eng->np)) || (rc = dev_upload(&d.udesc_w, eng->udesc_d))) return rc;
            if (eng->mma &&
                ((rc = dev_upload(&d.mma_kt, eng->mma_kt)) || (rc = dev_upload(&d.mma_kbase, eng->mma_kbase)) ||
                 (rc = dev_upload(&d.mma_wplan, eng->mma_wplan)) ||
                 (rc = dev_upload(&d.mma_desc, eng->mma_desc)) || (rc = dev_upload(&d.mma_dbase, eng->mma_dbase))))
                return rc;
            if (eng->mma)
                HIP_TRY(hipFuncSetAttribute(mma_kernel(eng), hipFuncAttributeMaxDynamicSharedMemorySize, (int)mma_lds(eng)));
            if (eng->mmt &&
                ((rc = dev_upload(&d.mmt_kt, eng->mmt_kt)) || (rc = dev_upload(&d.mmt_ktile, eng->mmt_ktile)) ||
                 (rc = dev_upload(&d.mmt_wplan, eng->mmt_wplan)) || (rc = dev_upload(&d.mmt_cidx, eng->mmt_cidx))))
                return rc;
            if (eng->mmt)
                HIP_TRY(hipFuncSetAttribute(mmt_kernel(eng), hipFuncAttributeMaxDynamicSharedMemorySize, (int)mmt_lds(eng)));
            if (eng->hs &&
                ((rc = dev_upload(&d.hs_kt, eng->hs_kt)) || (rc = dev_upload(&d.hs_cidx, eng->hs_cidx)) ||
                 (rc = dev_upload(&d.hs_pbase, eng->hs_pbase)) || (rc = dev_upload(&d.hs_ppos, eng->hs_ppos)) ||
                 (rc = dev_upload(&d.hs_dpos, eng->hs_dpos)) || (rc = dev_upload(&d.hs_dbase, eng->hs_dbase)) ||
                 (rc = dev_upload(&d.hs_pk, eng->hs_pk)) ||
                 (rc = dev_upload(&d.hs_wplan, eng->hs_wplan)) || (rc = dev_upload(&d.hs_pass, eng->hs_pass)) ||
                 (rc = dev_upload(&d.hs_dpk, eng->hs_dpk))))
                return rc;
            if (eng->hs)
                HIP_TRY(hipFuncSetAttribute(hs_kernel(eng), hipFuncAttributeMaxDynamicSharedMemorySize, (int)hs_lds(eng)));
            HIP_TRY(hipFuncSetAttribute((const void *)k_fwd_wide, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)wide_lds(eng)));
            return MDP_OK;
        }
        // (k_qrows' LDS attribute is set before its first launch and the
        // forward kernel loaded by set_grid_dev: nothing here loads a module)
    }
    return MDP_OK;
}

// k_qrows may take more than 64 KB of dynamic LDS: raise its limit once per
// device, just before its first launch
int qrows_attrs(const mdp_engine *eng, DevCtx &d)
{
    if (d.qrows_attr_set) return MDP_OK;
    const size_t lds_max = qrows_lds(eng, kQrowsMaxC);
    if (lds_max > 64 * 1024)
        for (const void *fn : {(const void *)k_qrows<8, true, 1>, (const void *)k_qrows<8, false, 1>,
                               (const void *)k_qrows<16, false, 1>, (const void *)k_qrows<24, false, 1>,
                               (const void *)k_qrows<8, true, 2>, (const void *)k_qrows<8, false, 2>,
                               (const void *)k_qrows<16, false, 2>, (const void *)k_qrows<8, true, 4>,
                               (const void *)k_qrows<8, false, 4>})
            HIP_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)std::min(lds_max, kQrowsLdsMax)));
    d.qrows_attr_set = true;
    return MDP_OK;
}

void free_device(DevCtx &d)
{
    (void)hipSetDevice(d.device);
    void *ptrs[] = {d.S, d.var_cols, d.row_col, d.pairA, d.pairB, d.pairOff, d.udesc, d.prog,
                    d.pairPart0, d.partP, d.partK0, d.e, d.c, d.ZPV, d.R, d.out, d.gpart,
                    d.zs, d.zsq, d.sv, d.Qrow, d.Zg, d.coltab, d.items, d.itemB, d.qstart, d.qitem,
                    d.Pg, d.V, d.np_d, d.udesc_w, d.zc, d.plist, d.qslot, d.qlane, d.islot,
                    d.mma_kt, d.mma_kbase, d.mma_desc, d.mma_dbase, d.mma_wplan,
                    d.mmt_kt, d.mmt_ktile, d.mmt_wplan, d.mmt_cidx,
                    d.hs_kt, d.hs_cidx, d.hs_pbase, d.hs_ppos, d.hs_dpos, d.hs_dbase, d.hs_pk,
                    d.hs_wplan, d.hs_pass, d.hs_dpk,
                    d.stamps[0], d.stamps[1], d.stamps[2]};
    for (void *ptr : ptrs)
        if (ptr) (void)hipFree(ptr);
    for (hipEvent_t ev : d.ev) (void)hipEventDestroy(ev);
    for (hipModule_t m : d.jit_mod)
        if (m) (void)hipModuleUnload(m);
    for (hipModule_t m : d.cmod) (void)hipModuleUnload(m);
    for (uint32_t *q : d.cqidx)
        if (q) (void)hipFree(q);
    if (d.vscr) (void)hipFree(d.vscr);
    if (d.stream) (void)hipStreamDestroy(d.stream);
}

// per-c coefficient stride: every forward use (deg+1 coefficients padded to
// an even count) plus two zero transitions of prefetch padding
size_t rsp_of(const mdp_engine *eng) { return (eng->deg + 2) & ~1u; }
size_t ldR_of(const mdp_engine *eng) { return ((size_t)eng->nuses + 2) * rsp_of(eng); }

// The point list of forward kernels with `epl` points per lane: the e rows
// whose ratio form is s (x < y, x = min(e, 1), y = 1 - x, as the kernel
// computes them), then those of form t, each run padded to a multiple of epl
// with duplicates of its last row (bit 31: computed, not stored), so every
// lane's points share one form and so their coefficient reads.  A sorted
// grid keeps its order (the kernels' stores stay coalesced).
std::vector<uint32_t> point_list(const double *e, uint32_t ne, uint32_t epl)
{
    std::vector<uint32_t> s_rows, t_rows;
    for (uint32_t i = 0; i < ne; ++i) {
        const double x = e[i] > 1.0 ? 1.0 : e[i], y = 1.0 - x;
        (x >= y ? t_rows : s_rows).push_back(i);
    }
    std::vector<uint32_t> pl;
    pl.reserve(ne + 2 * epl);
    for (const auto *rows : {&s_rows, &t_rows}) {
        pl.insert(pl.end(), rows->begin(), rows->end());
        while (!rows->empty() && pl.size() % epl) pl.push_back(rows->back() | 0x80000000u);
    }
    if (pl.empty()) pl.assign(epl, 0x80000000u);
    return pl;
}

int set_grid_dev(mdp_engine *eng, DevCtx &d, const double *e, uint32_t ne, const double *c,
                 uint32_t nc)
{
    // c < 0 is refused: the item factors are folded as |n_b - pC_b| (k_qrows
    // phase 2, k_witems, the fused prologue), which equals the reference's
    // (1 - piold)(1 - pC) + piold pC (main_MIDASPOM.c:40) only for pC >= 0;
    // at c < 0 the reference's pC = min(1, c S) is negative, not a probability
    // (and a NaN or infinite c: the pressures min(1, c S) are then clamped
    // by minNum, which drops NaN, where the reference would carry it)
    for (uint32_t i = 0; i < nc; ++i)
        if (!(c[i] >= 0.0) || std::isinf(c[i]))
            return mdp_set_error(MDP_EINVAL, "colonisation rate c[%u] = %g (the engine takes finite c >= 0)", i, c[i]);
    HIP_TRY(hipSetDevice(d.device));
    int rc;
    if ((rc = dev_reserve(&d.e, &d.cap_e, ne)) || (rc = dev_reserve(&d.c, &d.cap_c, nc))) return rc;
    d.ne_sform = 0;
    for (uint32_t i = 0; i < ne; ++i) {  // the kernels' form test: x = min(e, 1), s-form where x < 1 - x
        const double x = e[i] > 1.0 ? 1.0 : e[i];
        d.ne_sform += x < 1.0 - x;
    }
    const bool qglobal = eng->wide || eng->qglobal;  // Q rows from k_zrows + k_witems + k_wq
    if (eng->wide || eng->jit) {
        double cmax = eng->cbound;
        for (uint32_t i = 0; i < nc; ++i) cmax = std::isnan(c[i]) ? c[i] : std::max(cmax, std::fabs(c[i]));
        if ((rc = dev_reserve(&d.Qrow, &d.cap_qrow, (size_t)nc * eng->ldQ))) return rc;
        if (!(d.zs_cmax == cmax) && (rc = upload_qrows_tables(eng, d, cmax))) return rc;
    }
    if (qglobal) {
        if ((rc = dev_reserve(&d.Zg, &d.cap_zg, (size_t)nc * eng->nj + 1))) return rc;
        // k_zrows stages kZRows rows of explicit columns in dynamic LDS
        const size_t zl = (size_t)kZRows * d.zs_kmax * sizeof(double);
        if (zl > kQrowsLdsMax)
            return mdp_set_error(MDP_EUNSUPPORTED, "%u explicit colonisation columns per row exceed the LDS of k_zrows",
                                 d.zs_kmax);
        if (zl > 64 * 1024)
            HIP_TRY(hipFuncSetAttribute((const void *)k_zrows, hipFuncAttributeMaxDynamicSharedMemorySize, (int)zl));
        // c values per k_witems launch: item factors within kWidePgBytes
        const size_t cap_c = std::max<size_t>(1, std::min<size_t>(nc, 65535));
        d.wide_cb_items = (uint32_t)std::min(cap_c, std::max<size_t>(1, kWidePgBytes / 8 / std::max<size_t>(1, eng->nitems)));
        if (const char *cv = eng->opts.get("MDP_WIDE_CB"))  // tests: force several launches per slot
            d.wide_cb_items = std::min(d.wide_cb_items, (uint32_t)std::max(1, atoi(cv)));
        if (eng->hs) {  // k_fwd_hs reads the item factors of its columns: rows of nitems + 1 (zero slot)
            const size_t ldp = (size_t)eng->nitems + 1;
            d.wide_cb_items = (uint32_t)std::min<size_t>(nc, std::max<size_t>(1, kHsPgBytes / 8 / ldp));
            if (const char *cv = eng->opts.get("MDP_WIDE_CB"))
                d.wide_cb_items = std::min(d.wide_cb_items, (uint32_t)std::max(1, atoi(cv)));
            if ((rc = dev_reserve(&d.Pg, &d.cap_pg, (size_t)d.wide_cb_items * ldp))) return rc;
            HIP_TRY(hipMemset(d.Pg, 0, (size_t)d.wide_cb_items * ldp * sizeof(double)));
        } else if ((rc = dev_reserve(&d.Pg, &d.cap_pg, (size_t)d.wide_cb_items * eng->nitems + 1))) {
            return rc;
        }
    }
    if (eng->wide) {
        // c values per k_fwd_wide launch: the two state vectors of every
        // point of a launch within kWideVBytes (k_fwd_mma keeps them in LDS)
        const size_t ne_pad = (size_t)std::max<uint32_t>(1u, (ne + kBlock - 1) / kBlock) * kBlock;
        const size_t cap_c = std::max<size_t>(1, std::min<size_t>(nc, 65535));
        d.wide_cb_fwd = (uint32_t)std::min(cap_c, std::max<size_t>(1, kWideVBytes / 8 / (2 * (size_t)eng->npmax * ne_pad)));
        if (const char *cv = eng->opts.get("MDP_WIDE_CB"))
            d.wide_cb_fwd = std::min(d.wide_cb_fwd, (uint32_t)std::max(1, atoi(cv)));
        if (!eng->mma && !eng->mmt && (rc = dev_reserve(&d.V, &d.cap_v, 2 * (size_t)eng->npmax * d.wide_cb_fwd * ne_pad))) return rc;
    } else if (eng->jit) {
        // forward kernels with several points per lane read them from a list
        // that puts only e rows of one ratio form in a lane (spom_jit.cpp)
        const uint32_t epl_f = (uint32_t)eng->jit_epl;  // the fused variant's (jit_build: the reading variant's)
        const uint32_t epl_max = std::max<uint32_t>((uint32_t)eng->jit_epl, epl_f);
        d.plist_identity = true;
        if (epl_max > 1) {
            const std::vector<uint32_t> pl = point_list(e, ne, epl_max);
            for (uint32_t i = 0; i < pl.size() && d.plist_identity; ++i) d.plist_identity = pl[i] == i;
            if (!d.plist_identity) {  // an identity list is not uploaded: the kernels use the position
                if ((rc = dev_reserve(&d.plist, &d.cap_plist, pl.size()))) return rc;
                HIP_TRY(hipMemcpy(d.plist, pl.data(), pl.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
            }
            d.nlist = (uint32_t)pl.size();
        } else {
            d.nlist = ne;
        }
        d.nlist_epl = epl_max;
        // one e block per c column and a small per-c problem: the forward
        // kernel computes its column's Q itself (one launch); never for a
        // chunked series or Q rows built in HBM
        const uint32_t nl = eng->jit_epl > 1 ? d.nlist : ne;
        const uint32_t gy = (nl + eng->jit_kblock * eng->jit_epl - 1) / (eng->jit_kblock * eng->jit_epl);
        d.fused = eng->chunks.empty() && !eng->qglobal && !eng->jit_plan.vlds && fused_lds(eng, d.ct_len) <= kFusedLdsMax &&
                  d.zs_kmax <= eng->jit_plan.kzmax && (eng->fused_mode == 1 || (eng->fused_mode == -1 && gy <= 1));
        // a column of a tall grid (an even number of e blocks, so no lane more
        // idles) in half the blocks of twice the threads: each block stages
        // its column's Q row once (config 3: forward 45.7-46.9 -> 44.3 us) --
        // while that still leaves a block for every CU (a column slab of
        // config 3, 1 024 x 128: 128 tall blocks would idle half the chip)
        if (!d.ncu) {
            int v = 0;
            d.ncu = hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d.device) == hipSuccess && v > 0
                        ? (uint32_t)v : 256u;
        }
        d.tall = !d.fused && eng->chunks.empty() && !eng->jit_plan.vlds && !eng->jit_shape_env &&
                 eng->jit_kblock * 2 == (uint32_t)kJitKblockTall && gy >= 2 && gy % 2 == 0 &&
                 (uint64_t)nc * (gy / 2) >= d.ncu;
        if ((rc = jit_load(eng, d, d.fused ? 1 : d.tall ? 2 : 0))) return rc;
        if (!eng->chunks.empty()) {  // the state vectors handed between chunks
            d.ldv = gy * eng->jit_kblock * (uint32_t)eng->jit_epl;
            uint32_t nb = 1;  // most states at a chunk boundary
            for (size_t i = 1; i < eng->chunks.size(); ++i) nb = std::max(nb, eng->chunks[i].np[0]);
            if ((rc = dev_reserve(&d.vscr, &d.cap_vscr, (size_t)nb * nc * d.ldv))) return rc;
        }
        // c values per k_qrows workgroup: enough workgroups for every CU, within the LDS
        uint32_t cb = nc >= 1024 ? 4u : nc >= 512 ? 2u : 1u;  // power of two
        cb = std::min(cb, eng->nvar <= 8 ? 4u : eng->nvar <= 16 ? 2u : 1u);  // registers (k_qrows)
        while (cb > 1 && qrows_lds(eng, cb) > kQrowsLdsMax) cb >>= 1;
        d.qrows_cb = cb;
    } else if ((rc = dev_reserve(&d.ZPV, &d.cap_zpv, (size_t)nc * (eng->nvar + 1) * eng->nstates)) ||
               (rc = dev_reserve(&d.R, &d.cap_r, (size_t)nc * ldR_of(eng)))) {
        return rc;
    }
    if (!eng->jit && !eng->wide && !eng->lds_part &&
        (rc = dev_reserve(&d.gpart, &d.cap_gpart, (size_t)nc * eng->partP.size() * (eng->nvar + 1))))
        return rc;
    if (eng->diag) {
        d.nst[0] = eng->jit ? (size_t)nc
                            : (size_t)((eng->nstates + kZpvJ - 1) / kZpvJ) * ((nc + kZpvCT - 1) / kZpvCT);
        d.nst[1] = nc;
        d.nst[2] = (size_t)nc * ((ne + kBlock - 1) / kBlock);  // >= the JIT grid (EPL >= 1)
        for (int k = 0; k < 3; ++k) {
            if ((rc = dev_reserve(&d.stamps[k], &d.cap_st[k], d.nst[k] * kStampSlots))) return rc;
            HIP_TRY(hipMemset(d.stamps[k], 0, d.cap_st[k] * sizeof(unsigned long long)));
        }
    }
    if (ne) HIP_TRY(hipMemcpy(d.e, e, ne * sizeof(double), hipMemcpyHostToDevice));
    if (nc) HIP_TRY(hipMemcpy(d.c, c, nc * sizeof(double), hipMemcpyHostToDevice));
    d.ne = ne;
    d.nc = nc;
    return MDP_OK;
}

template <int NP, int DEG, int EPL>
void launch_fwd_epl(const mdp_engine *eng, const DevCtx &d, double *out, OutStrides os, hipStream_t s)
{
    uint32_t se = os.se, sc = os.sc;
    dim3 grid(d.nc, (d.ne + kBlock * EPL - 1) / (kBlock * EPL));
    const uint32_t nprog = (uint32_t)eng->prog.size() - 1;
    note_launch(eng, "%s<%d,%d,%d>", eng->fwd_lds ? "k_forward_lds" : "k_forward", NP, DEG, EPL);
    if (eng->fwd_lds)
        MDP_LAUNCH((k_forward_lds<NP, DEG, EPL>), grid, dim3(kBlock), eng->fwd_lds_bytes, s,
                           d.R, ldR_of(eng), d.prog, nprog, eng->np[0], eng->prior0, d.e, d.ne, out, se,
                           sc, d.stamps[2]);
    else
        MDP_LAUNCH((k_forward<NP, DEG, EPL>), grid, dim3(kBlock), 0, s, d.R, ldR_of(eng),
                           d.prog, nprog, eng->np[0], eng->prior0, d.e, d.ne, out, se, sc);
}

template <int NP, int DEG>
void launch_fwd(const mdp_engine *eng, const DevCtx &d, double *out, OutStrides os, hipStream_t s)
{
    if constexpr (NP <= 4 && DEG <= 8) {
        if (eng->epl == 1) return launch_fwd_epl<NP, DEG, 1>(eng, d, out, os, s);
        if (eng->epl == 4) return launch_fwd_epl<NP, DEG, 4>(eng, d, out, os, s);
    }
    launch_fwd_epl<NP, DEG, kEPL>(eng, d, out, os, s);
}

template <int NP>
int launch_fwd_deg(const mdp_engine *eng, const DevCtx &d, double *out, OutStrides os, hipStream_t s)
{
    switch (eng->deg) {
    case 4: launch_fwd<NP, 4>(eng, d, out, os, s); break;
    case 8: launch_fwd<NP, 8>(eng, d, out, os, s); break;
    case 16: launch_fwd<NP, 16>(eng, d, out, os, s); break;
    case 24: launch_fwd<NP, 24>(eng, d, out, os, s); break;
    default: return mdp_set_error(MDP_EUNSUPPORTED, "no forward kernel for degree %u", eng->deg);
    }
    return MDP_OK;
}

int launch_forward(const mdp_engine *eng, const DevCtx &d, double *out, OutStrides os, hipStream_t s)
{
    int rc;
    if (eng->jit) {
        const double *Qrow = d.Qrow;
        double prior0 = eng->prior0;
        const double *ev = d.e;
        uint32_t ne = d.ne, nc = d.nc, one = 1;
        unsigned long long *st = d.stamps[2];
        const double *cv = d.c, *ctab = d.coltab;
        uint32_t ctl = d.ct_len, kmax = d.zs_kmax;
        double *vscr = d.vscr;
        uint32_t ldv = d.ldv;
        const uint32_t *qidx = nullptr;
        uint32_t se = os.se, sc = os.sc;
        // threads per e block: kb (x 2 with the split state-vector kernel)
        const uint32_t kb = d.fused ? eng->jit_kblock_fused : d.tall ? (uint32_t)kJitKblockTall : eng->jit_kblock;
        const uint32_t pro = d.fused ? eng->jit_pro_fused : 1u;
        const uint32_t epl = d.fused ? (uint32_t)eng->jit_epl_fused : (uint32_t)eng->jit_epl;
        const uint32_t spl = eng->jit_plan.vlds && (eng->jit_plan.vsplit == 2 || eng->jit_plan.vsplit == 4)
                                 ? (uint32_t)eng->jit_plan.vsplit : 1u;
        // several points per lane: the grid's point list (set_grid_dev)
        const uint32_t *plist = epl > 1 && !d.plist_identity ? d.plist : nullptr;
        uint32_t nlist = epl > 1 ? d.nlist : d.ne;
        if (epl > 1 && ((!plist && !d.plist_identity) || d.nlist_epl % epl))
            return mdp_set_error(MDP_EINVAL, "no point list for %u points per lane", epl);
        void *args[] = {(void *)&Qrow, (void *)&prior0, (void *)&ev,  (void *)&ne,   (void *)&nc,
                        (void *)&out,  (void *)&se,     (void *)&one, (void *)&st,   (void *)&cv,
                        (void *)&ctab, (void *)&ctl,    (void *)&kmax, (void *)&vscr, (void *)&ldv,
                        (void *)&qidx, (void *)&sc,     (void *)&plist, (void *)&nlist};
        const uint64_t gy = (nlist + kb * epl - 1) / (kb * epl);
        const uint32_t fc = d.fused ? (uint32_t)eng->jit_plan.fused_cols : 1u;
        const uint64_t nb = gy * ((d.nc + fc - 1) / fc);  // e blocks x column groups
        if (nb * kb * fc * spl > 0xffffffffull)
            return mdp_set_error(MDP_EUNSUPPORTED, "grid %u x %u too large", d.ne, d.nc);
        if (!eng->chunks.empty()) {  // a long series: its chunks in order on the stream
            const size_t nch = d.cfn.size();
            if (nch != eng->chunks.size() || d.cqidx.size() != nch)
                return mdp_set_error(MDP_EHIP, "forward chunks not loaded (%zu of %zu)", nch, eng->chunks.size());
            for (size_t i = 0; i < nch; ++i) {
                qidx = d.cqidx[i];
                HIP_TRY(hipExtModuleLaunchKernel(d.cfn[i], (uint32_t)(nb * kb * spl), 1, 1, kb * spl, 1, 1, 0, s, args,
                                                 nullptr, i == 0 ? t_kev.start : nullptr,
                                                 i + 1 == nch ? t_kev.stop : nullptr, 0));
            }
            note_launch(eng, "mdp_fwd_jit<reading,maxA%u,chunks%zu%s>", eng->maxA, nch,
                        eng->chunks[0].qidx.empty() ? "" : ",gather");
            return MDP_OK;
        }
        const uint32_t dyn = d.fused ? (d.ct_len + 2) * (uint32_t)sizeof(double) : 0u;  // + staging scratch
        HIP_TRY(hipExtModuleLaunchKernel(d.jit_fn[d.fused ? 1 : d.tall ? 2 : 0], (uint32_t)(nb * kb * fc * spl * pro), 1, 1,
                                         kb * fc * spl * pro, 1, 1, dyn, s, args, nullptr, t_kev.start, t_kev.stop, 0));
        note_launch(eng, "mdp_fwd_jit<%s,maxA%u>", d.fused ? "fused" : "reading", eng->maxA);
        if (d.tall) note_launch(eng, "mdp_fwd_jit<reading,kb%d>", kJitKblockTall);
        return MDP_OK;
    }
    switch (eng->variant / 100) {
    case 1: rc = launch_fwd_deg<1>(eng, d, out, os, s); break;
    case 2: rc = launch_fwd_deg<2>(eng, d, out, os, s); break;
    case 4: rc = launch_fwd_deg<4>(eng, d, out, os, s); break;
    case 8: rc = launch_fwd_deg<8>(eng, d, out, os, s); break;
    case 16: rc = launch_fwd_deg<16>(eng, d, out, os, s); break;
    default: return mdp_set_error(MDP_EUNSUPPORTED, "no forward kernel variant %u", eng->variant);
    }
    if (rc) return rc;
    HIP_TRY(hipGetLastError());
    return MDP_OK;
}

template <bool LDSZ, bool LDSP, int NV>
void launch_coefs_nv(const mdp_engine *eng, const DevCtx &d, hipStream_t s)
{
    note_launch(eng, "k_coefs<%d,%d,%d>", (int)LDSZ, (int)LDSP, NV);
    MDP_LAUNCH((k_coefs<LDSZ, LDSP, NV>), dim3(d.nc), dim3(kBlock), eng->coef_lds, s, d.ZPV,
                       eng->nstates, eng->nvar, d.pairA, d.pairB, d.pairOff, d.pairPart0, eng->npairs,
                       d.partP, d.partK0, (uint32_t)eng->partP.size(), eng->ncoef, d.udesc,
                       eng->nuses, eng->deg, d.R, ldR_of(eng), d.gpart, d.stamps[1]);
}

template <bool LDSZ, bool LDSP>
void launch_coefs_lds(const mdp_engine *eng, const DevCtx &d, hipStream_t s)
{
    const uint32_t nv = eng->nvar;
    if (nv <= 8) launch_coefs_nv<LDSZ, LDSP, 8>(eng, d, s);
    else if (nv <= 16) launch_coefs_nv<LDSZ, LDSP, 16>(eng, d, s);
    else launch_coefs_nv<LDSZ, LDSP, 24>(eng, d, s);
}

int launch_coefs(const mdp_engine *eng, const DevCtx &d, hipStream_t s)
{
    if (eng->lds_zpv) launch_coefs_lds<true, true>(eng, d, s);
    else if (eng->lds_part) launch_coefs_lds<false, true>(eng, d, s);
    else launch_coefs_lds<false, false>(eng, d, s);
    HIP_TRY(hipGetLastError());
    return MDP_OK;
}

// Wide path, slot 1 (k_witems + k_wq per chunk of c values) or slot 2
// (k_fwd_wide per chunk).  A profiled run times the slot as a whole: events
// recorded around its launches.
int launch_wide(const mdp_engine *eng, const DevCtx &d, int k, double *out, OutStrides os, hipStream_t s)
{
    const KernelEvents ev = t_kev;
    t_kev = KernelEvents{};
    if (ev.start) HIP_TRY(hipEventRecord(ev.start, s));
    auto witems = [&](uint32_t c0, uint32_t n, uint32_t ldp) {
        const dim3 gi((eng->nitems + kBlock - 1) / kBlock, n);
#define MDP_WITEMS(NV) \
    do { note_launch(eng, "k_witems<%d>", NV); \
    hipLaunchKernelGGL((k_witems<NV>), gi, dim3(kBlock), 0, s, d.c, d.nc, c0, eng->nvar, d.Zg, d.sv, eng->nitems, d.items, d.Pg, ldp); } while (0)
        if (eng->nvar <= 8) MDP_WITEMS(8);
        else if (eng->nvar <= 16) MDP_WITEMS(16);
        else MDP_WITEMS(24);
#undef MDP_WITEMS
    };
    if (eng->hs) {
        // slot 1: the item factors of every column when they fit one Pg
        // block (kHsPgBytes), else nothing; slot 2: k_fwd_hs, or per column
        // chunk k_witems then k_fwd_hs
        const uint32_t cb = d.wide_cb_items, ldp = eng->nitems + 1;
        const bool one = cb >= d.nc;
        if (k == 1) {
            if (one && eng->nitems) witems(0, d.nc, ldp);
        } else {
            const uint32_t rt = eng->hs_rt, nb = eng->hs_nb, npb = (d.ne + mmt_pts(rt) - 1) / mmt_pts(rt);
            for (uint32_t c0 = 0; c0 < d.nc; c0 += cb) {
                const uint32_t n = std::min(cb, d.nc - c0);
                if (!one && eng->nitems) witems(c0, n, ldp);
                const uint64_t nbk = (uint64_t)npb * n;
                if (nbk > 0x7fffffffull) return mdp_set_error(MDP_EUNSUPPORTED, "grid of %llu k_fwd_hs workgroups", (unsigned long long)nbk);
                note_launch(eng, "k_fwd_hs<%u,%u>", rt, nb);
#define MDP_HS(RT, NB, NW) \
    hipLaunchKernelGGL((k_fwd_hs<RT, NB, NW>), dim3((uint32_t)nbk), dim3(NW * 64), hs_lds(eng), s, d.Pg, ldp, c0, d.np_d, \
                       d.hs_kt, d.hs_cidx, d.hs_wplan, d.hs_pass, d.hs_pbase, d.hs_ppos, d.hs_dpos, \
                       d.hs_dbase, d.hs_dpk, d.hs_pk, eng->tmax, eng->prior0, d.e, d.ne, out, os.se, os.sc, eng->hs_probe)
                if (nb == 8 && eng->hs_nw == 8) MDP_HS(2, 8, 8);
                else if (nb == 8) MDP_HS(4, 8, 16);
                else if (nb == 9) MDP_HS(2, 9, 16);
                else MDP_HS(1, 10, 16);
#undef MDP_HS
            }
        }
    } else if (k == 1) {
        const uint32_t cb = d.wide_cb_items;
        for (uint32_t c0 = 0; c0 < d.nc; c0 += cb) {
            const uint32_t n = std::min(cb, d.nc - c0);
            witems(c0, n, eng->nitems);
            const dim3 gq((uint32_t)((eng->ldQ + kBlock - 1) / kBlock), n);
            note_launch(eng, "k_wq");
            hipLaunchKernelGGL(k_wq, gq, dim3(kBlock), 0, s, c0, eng->nitems, d.Pg, eng->ncoef_d, d.qstart, d.qitem,
                               d.Qrow, (uint32_t)eng->ldQ);
        }
    } else if (eng->mmt) {  // the matrix-core forward: every c in one launch, blocks dealt XCD-aware
        const uint32_t rt = eng->mmt_rt, rows = eng->mmt_rows, npb = (d.ne + mmt_pts(rt) - 1) / mmt_pts(rt);
        const bool db = mmt_shape(eng).db;
        const uint64_t nb = (uint64_t)npb * d.nc;
        if (nb > 0x7fffffffull) return mdp_set_error(MDP_EUNSUPPORTED, "grid of %llu k_fwd_mmt workgroups", (unsigned long long)nb);
        note_launch(eng, "k_fwd_mmt<%u,%u,%s>", rt, rows, db ? "2buf" : "1buf");
#define MDP_MMT(RT, ROWS, DB) \
    hipLaunchKernelGGL((k_fwd_mmt<RT, ROWS, DB>), dim3((uint32_t)nb), dim3(kMmaThreads), mmt_lds(eng), s, d.Qrow, (uint32_t)eng->ldQ, \
                       d.np_d, d.mmt_kt, d.mmt_cidx, d.mmt_ktile, d.mmt_wplan, eng->tmax, eng->prior0, d.e, d.ne, \
                       eng->maxA, out, os.se, os.sc)
        if (rows == 128) MDP_MMT(4, 128, true);
        else if (rows == 256) MDP_MMT(2, 256, false);
        else if (rows == 512) MDP_MMT(2, 512, false);
        else MDP_MMT(1, 1024, false);
#undef MDP_MMT
    } else if (eng->mma) {  // round 5's matrix-core forward (MDP_WIDE_MMA=1; years of up to 256 states)
        uint32_t se = os.se, sc = os.sc;
        for (uint32_t c0 = 0; c0 < d.nc; c0 += 65535) {
            const uint32_t n = std::min(65535u, d.nc - c0);
            const uint32_t pts = mma_pts(eng->mma_npm);
            const dim3 g((d.ne + pts - 1) / pts, n);
            note_launch(eng, "k_fwd_mma<%u>", eng->mma_npm);
#define MDP_MMA(NPM) \
    hipLaunchKernelGGL((k_fwd_mma<NPM>), g, dim3(kMmaThreads), mma_lds(eng), s, d.Qrow, (uint32_t)eng->ldQ, d.np_d, \
                       d.mma_kt, d.mma_kbase, d.mma_desc, d.mma_dbase, d.mma_wplan, eng->tmax, eng->prior0, d.e, d.ne, c0, eng->maxA, \
                       eng->mma_ktmax, eng->ncoef_d, out, se, sc)
            if (eng->mma_npm == 64) MDP_MMA(64);
            else if (eng->mma_npm == 128) MDP_MMA(128);
            else MDP_MMA(256);
#undef MDP_MMA
        }
    } else {
        const uint32_t cb = d.wide_cb_fwd;
        uint32_t se = os.se, sc = os.sc;
        for (uint32_t c0 = 0; c0 < d.nc; c0 += cb) {
            const uint32_t n = std::min(cb, d.nc - c0);
            const dim3 g((d.ne + kBlock - 1) / kBlock, n);
            note_launch(eng, "k_fwd_wide");
            hipLaunchKernelGGL(k_fwd_wide, g, dim3(kBlock), wide_lds(eng), s, d.Qrow, (uint32_t)eng->ldQ, d.udesc_w,
                               d.np_d, eng->tmax, eng->prior0, d.e, d.ne, c0, eng->maxA, d.V, eng->npmax, out, se, sc);
        }
    }
    HIP_TRY(hipGetLastError());
    if (ev.stop) HIP_TRY(hipEventRecord(ev.stop, s));
    return MDP_OK;
}

// Does kernel slot k (0: Q rows / k_zpv, 1: k_coefs, 2: forward) run on this path?
bool slot_active(const mdp_engine *eng, const DevCtx &d, int k)
{
    if (eng->wide || (eng->jit && eng->qglobal)) return k == 2 || eng->nitems;
    // the direct path computes its Z rows inside k_qrows (slot 0 idle); the
    // wide path (and Q rows built in HBM) keeps k_zrows for its item kernel
    if (eng->jit) return k == 2 || (k == 1 && eng->nitems && !d.fused);
    return k != 1 || eng->nuses;
}

int launch_slot(mdp_engine *eng, DevCtx &d, int k, double *out, OutStrides os, hipStream_t s)
{
    if (!slot_active(eng, d, k)) return MDP_OK;
    if ((eng->wide && k > 0) || (eng->jit && eng->qglobal && k == 1)) return launch_wide(eng, d, k, out, os, s);
    if (k == 2) return launch_forward(eng, d, out, os, s);
    if ((eng->jit || eng->wide) && k == 0) {  // Z rows
        const uint32_t kmax = d.zs_kmax;
        const dim3 grid((d.nc + 64 * kZC - 1) / (64 * kZC), (eng->nj + kZRows - 1) / kZRows);
        note_launch(eng, "k_zrows");
        MDP_LAUNCH(k_zrows, grid, dim3(kBlock), (size_t)kZRows * kmax * sizeof(double), s, d.c, d.nc, eng->nj,
                   kmax, d.zs, d.zc, d.Zg);
        HIP_TRY(hipGetLastError());
        return MDP_OK;
    }
    if (eng->jit) {  // k == 1: Q rows
        if (int rc = qrows_attrs(eng, d)) return rc;
        const uint32_t cb = d.qrows_cb;
        const dim3 grid((d.nc + cb - 1) / cb);
        const size_t lds = qrows_lds(eng, cb);
#define MDP_QROWS_CB(NV, EX, CB)                                                                        \
    do {                                                                                                \
    note_launch(eng, "k_qrows<%d,%d,%d>", NV, (int)EX, CB);                                              \
    MDP_LAUNCH((k_qrows<NV, EX, CB>), grid, dim3(kQrowsBlock), lds, s, d.c, d.nc, eng->nvar, eng->nj,         \
               d.zs_kmax, d.zsq, d.zc, d.sv, eng->nitems, d.items, eng->ncoef_d, d.qstart,                     \
               (uint32_t)eng->qitem.size(), d.qitem, d.Qrow, (uint32_t)eng->ldQ, d.stamps[1],                 \
               (uint32_t)(eng->qrows_xcd ? 1u : 0u), d.qslot, (uint32_t)eng->qslot.size(), eng->qslot_lglmax,   \
               (const uint4 *)d.qlane, d.islot, eng->npl_slots); } while (0)
        // c values per workgroup: <= qrows_maxcb(nvar) (register budget at 1024 threads)
        if (eng->nvar == 8) {
            if (cb == 4) MDP_QROWS_CB(8, true, 4);
            else if (cb == 2) MDP_QROWS_CB(8, true, 2);
            else MDP_QROWS_CB(8, true, 1);
        } else if (eng->nvar < 8) {
            if (cb == 4) MDP_QROWS_CB(8, false, 4);
            else if (cb == 2) MDP_QROWS_CB(8, false, 2);
            else MDP_QROWS_CB(8, false, 1);
        } else if (eng->nvar <= 16) {
            if (cb == 2) MDP_QROWS_CB(16, false, 2);
            else MDP_QROWS_CB(16, false, 1);
        } else {
            MDP_QROWS_CB(24, false, 1);
        }
#undef MDP_QROWS_CB
        HIP_TRY(hipGetLastError());
        return MDP_OK;
    }
    if (k == 0) {
        dim3 grid((eng->nstates + kZpvJ - 1) / kZpvJ, (d.nc + kZpvCT - 1) / kZpvCT);
        note_launch(eng, "k_zpv");
        MDP_LAUNCH(k_zpv, grid, dim3(kBlock), 0, s, d.S, eng->nstates, eng->n - eng->nvar, eng->nvar, d.c,
                   d.nc, d.ZPV, d.stamps[0]);
        HIP_TRY(hipGetLastError());
        return MDP_OK;
    }
    return launch_coefs(eng, d, s);
}

int run_dev(mdp_engine *eng, DevCtx &d, double *out, OutStrides os, hipStream_t s)
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
        d.ev_mask.resize(d.ev_used);
        d.ev_mask.back() = 0;
    }
    struct Reset {
        ~Reset() { t_kev = KernelEvents{}; }
    } reset;
    for (int k = 0; k < 3; ++k) {
        if (!slot_active(eng, d, k)) continue;
        // only launched kernels carry events (no marker packets between kernels)
        t_kev = prof ? KernelEvents{ev[2 * k], ev[2 * k + 1]} : KernelEvents{};
        if (prof) d.ev_mask.back() |= (uint8_t)(1u << k);
        int rc = launch_slot(eng, d, k, out, os, s);
        if (rc) return rc;
    }
    return MDP_OK;
}

// Mean duration of each kernel of the run: one full run, then every kernel
// launched `reps` times back to back between two events on the stream (no
// per-launch events, so the figure is the kernel's own, as rocprofv3 sees it).
int time_kernels(mdp_engine *eng, DevCtx &d, double *out, OutStrides os, hipStream_t s, int reps, double *ms)
{
    int rc = run_dev(eng, d, out, os, s);
    if (rc) return rc;
    hipEvent_t a, b;
    HIP_TRY(hipEventCreate(&a));
    HIP_TRY(hipEventCreate(&b));
    for (int k = 0; k < 3; ++k) {
        ms[k] = 0.0;
        if (!slot_active(eng, d, k)) continue;
        if ((rc = launch_slot(eng, d, k, out, os, s))) break;  // warm
        (void)hipEventRecord(a, s);
        for (int r = 0; r < reps && !rc; ++r) rc = launch_slot(eng, d, k, out, os, s);
        (void)hipEventRecord(b, s);
        if (rc) break;
        float t = 0;
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&t, a, b);
        ms[k] = t / reps;
    }
    // leave the output as a full run computes it
    if (!rc) rc = run_dev(eng, d, out, os, s);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return rc;
}

// Mean kernel durations over every profiled run since the last collect.
int collect_times(mdp_engine *eng, DevCtx &d)
{
    if (d.ev_used == 0) return MDP_OK;
    HIP_TRY(hipSetDevice(d.device));
    HIP_TRY(hipEventSynchronize(d.ev[(d.ev_used - 1) * kNumEv + kNumEv - 1]));
    double sum[3] = {0, 0, 0};
    size_t cnt[3] = {0, 0, 0};
    for (size_t r = 0; r < d.ev_used; ++r)
        for (int k = 0; k < 3; ++k) {
            if (!((d.ev_mask[r] >> k) & 1u)) continue;
            float ms = 0;
            HIP_TRY(hipEventElapsedTime(&ms, d.ev[r * kNumEv + 2 * k], d.ev[r * kNumEv + 2 * k + 1]));
            sum[k] += ms;
            ++cnt[k];
        }
    for (int k = 0; k < 3; ++k) eng->last_ms[k] = cnt[k] ? sum[k] / (double)cnt[k] : 0.0;
    eng->nlast = 3;
    eng->runs_collected = d.ev_used;
    d.ev_used = 0;
    return MDP_OK;
}

// Split a long series into chunks of whole years for the hipRTC forward
// kernel: at most `U` uses per chunk (straight-line code stays a bounded
// size), preferring a boundary year with one state (the smallest hand-over)
// in the last quarter of a chunk.  With `gather`, each chunk stages only the
// Q groups its uses read (at most kJitChunkQ doubles, a chunk-local layout of
// even-aligned groups) instead of the whole Q row.
int plan_chunks(mdp_engine *eng, uint32_t U, bool gather, size_t qlimit)
{
    const MdpJitPlan &base = eng->jit_plan;
    const std::vector<uint32_t> &np = eng->np;
    const std::vector<uint32_t> &ud = eng->udesc_d;
    const uint32_t T = eng->tmax;
    const int epl = base.epl > 0 ? base.epl : mdp_jit_default_epl(ud);
    auto gsize = [](uint32_t d) { return (((d >> kOffBits) & 31u) + 2u) & ~1u; };  // nX + 1, even
    eng->chunks.clear();
    uint32_t t0 = 0;
    size_t u0 = 0;
    uint32_t e0 = 0;  // pending exponent of B at the chunk boundary (spom_jit.cpp)
    while (t0 + 1 < T) {
        size_t cur = 0, qloc = 0, u1 = u0, best_u1 = 0;
        uint32_t t1 = t0, best_t1 = 0;
        std::set<uint32_t> loc;
        while (t1 + 1 < T) {
            const size_t nu = (size_t)np[t1] * np[t1 + 1];
            size_t addq = 0;
            std::set<uint32_t> fresh;
            if (gather)
                for (size_t u = u1; u < u1 + nu; ++u) {
                    const uint32_t off = ud[u] & kOffMask;
                    if (!loc.count(off) && fresh.insert(off).second) addq += gsize(ud[u]);
                }
            if (cur > 0 && (cur + nu > U || (gather && qloc + addq > qlimit))) break;
            cur += nu;
            qloc += addq;
            loc.insert(fresh.begin(), fresh.end());
            u1 += nu;
            ++t1;
            if (np[t1] == 1 && 4 * cur >= 3 * (size_t)U) {
                best_t1 = t1;
                best_u1 = u1;
            }
        }
        if (t1 + 1 < T && best_t1 && best_t1 < t1) {
            t1 = best_t1;
            u1 = best_u1;
        }
        MdpJitPlan c = base;
        c.fused = false;
        c.epl = epl;
        c.np.assign(np.begin() + t0, np.begin() + t1 + 1);
        c.udesc.assign(ud.begin() + u0, ud.begin() + u1);
        c.first = t0 == 0;
        c.last = t1 + 1 == T;
        c.e0 = e0;
        e0 = mdp_jit_end_exp(c);
        if (gather) {  // chunk-local Q layout, groups in first-use order
            std::map<uint32_t, uint32_t> lo;
            c.qidx.clear();
            for (uint32_t &d : c.udesc) {
                const uint32_t off = d & kOffMask;
                auto it = lo.find(off);
                if (it == lo.end()) {
                    it = lo.emplace(off, (uint32_t)c.qidx.size()).first;
                    for (uint32_t m = 0; m < gsize(d); ++m) c.qidx.push_back(off + std::min(m, (d >> kOffBits) & 31u));
                }
                d = (d & ~kOffMask) | it->second;
            }
            c.ldq_row = base.ldQ;
        }
        eng->chunks.push_back(std::move(c));
        t0 = t1;
        u0 = u1;
    }
    return eng->chunks.empty() ? mdp_set_error(MDP_EUNSUPPORTED, "no forward chunks") : MDP_OK;
}

}  // namespace

extern "C" {

int mdp_engine_create(const mdp_problem *p, const int *devices, int n_devices, mdp_engine **out)
{
    return mdp_engine_create_opts(p, devices, n_devices, nullptr, out);
}

int mdp_engine_create_opts(const mdp_problem *p, const int *devices, int n_devices, const char *options,
                           mdp_engine **out)
{
    if (!p || !out || n_devices < 0) return mdp_set_error(MDP_EINVAL, "null argument");
    *out = nullptr;
    // MDP_SETUP_TIMING=1: the set-up's split on stderr (planning, hipRTC /
    // code-object cache, device set-up)
    const bool st_on = getenv("MDP_SETUP_TIMING") && atoi(getenv("MDP_SETUP_TIMING")) != 0;
    auto st_now = []() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double st0 = st_now();
    double st_jit0 = st0, st_jit1 = st0;
    EngineOpts opts;
    if (int orc = parse_engine_opts(options, opts)) return orc;
    if (p->n == 0 || p->tmax == 0 || !p->M || !p->year_off || !p->year_ids || !p->prior ||
        !p->short_state || (p->nvar && !p->var_cols))
        return mdp_set_error(MDP_EINVAL, "incomplete problem description");
    int ndev = 0;
    // MDP_JIT_CHECK=1 without a device: plan and compile both forward
    // variants (hipRTC runs offline), then report MDP_ENODEV -- the CPU
    // test that the generated sources compile for gfx950
    const char *jcheck = opts.get("MDP_JIT_CHECK");
    const bool jit_check = jcheck && atoi(jcheck) != 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        ndev = 0;
        if (!jit_check) return mdp_set_error(MDP_ENODEV, "no HIP device available");
    }
    mdp_engine *eng = new (std::nothrow) mdp_engine();
    if (!eng) return mdp_set_error(MDP_ENOMEM, "out of host memory");
    eng->opts = std::move(opts);
    int rc = build_plan(eng, p);
    if (rc) {
        delete eng;
        return rc;
    }
    eng->fwd_lds_bytes = ldR_of(eng) * sizeof(double) + (eng->prog.size() + 1) * sizeof(uint32_t);
    eng->fwd_lds = eng->fwd_lds_bytes <= kFwdLds;
    if (const char *ev = eng->opts.get("MDP_FWD"))
        if (!strcmp(ev, "scalar")) eng->fwd_lds = false;
    if (const char *ev = eng->opts.get("MDP_EPL")) {
        const int v = atoi(ev);
        if (v == 1 || v == 2 || v == 4) eng->epl = v;
    }
    if (const char *ev = eng->opts.get("MDP_DIAG")) eng->diag = atoi(ev) != 0;
    {
        const char *jv = eng->opts.get("MDP_JIT");
        const bool jit_off = jv && !strcmp(jv, "0");
        // years of 17-64 states: the specialised forward kernel with its
        // state vectors in LDS (plan.vlds), unless the series is so long that
        // hipRTC would take minutes; MDP_WIDE=1 forces the wide kernels
        const char *wv0 = eng->opts.get("MDP_WIDE");
        const bool wide_forced = wv0 && atoi(wv0) != 0;
        bool vlds = false;
        uint32_t vlds_max_uses = kVldsMaxUses;
        if (const char *mv = eng->opts.get("MDP_VLDS_MAXUSES")) vlds_max_uses = (uint32_t)std::max(0, atoi(mv));
        const uint32_t vkb = kBlock;  // points per workgroup (their states: npmax x vkb doubles of LDS)
        if (eng->wide && !wide_forced && !jit_off && eng->npmax <= kVldsMaxStates && eng->nuses <= vlds_max_uses) {
            eng->wide = false;
            vlds = true;
        }
        const bool want = !eng->wide && !jit_off;
        bool want_jit = want && build_direct_plan(eng, p) == MDP_OK;
        // k_qrows keeps every table of its c values in LDS; larger problems
        // build their Q rows in HBM (k_zrows + k_witems + k_wq, the same bits)
        const char *qg = eng->opts.get("MDP_QGLOBAL");
        eng->qglobal = want_jit && (qrows_lds(eng, 1) > kQrowsLdsMax || (qg && atoi(qg) != 0));
        eng->ldQ = ((size_t)eng->ncoef_d + 1) & ~(size_t)1;
        // a series longer than kJitMaxUses uses (or a Q row past the LDS) runs
        // as chunks of years (MDP_JIT_CHUNK / MDP_JIT_GATHER force them)
        uint32_t chunk_uses = kJitChunkUses;
        const char *cv = eng->opts.get("MDP_JIT_CHUNK");
        if (cv) chunk_uses = (uint32_t)std::max(1, atoi(cv));
        const char *gv = eng->opts.get("MDP_JIT_GATHER");
        // coefficients a forward kernel may stage: what the LDS leaves beside
        // the wide years' state vectors (npmax x 256 lanes) when they are there
        // (halved: the forward kernel keeps each Q row twice, in stored and in
        // reversed group order -- spom_jit.cpp, the ratio forms)
        const size_t qlimit = (vlds ? std::min(kJitChunkQ, (kQrowsLdsMax - (size_t)eng->npmax * vkb * sizeof(double) -
                                                          2048) / sizeof(double))
                                    : kJitChunkQ) / 2;
        const bool gather = eng->ldQ > qlimit || (gv && atoi(gv) != 0);
        const bool chunked = eng->nuses > kJitMaxUses || gather || (cv && eng->nuses > chunk_uses);
        if (want_jit && eng->nuses > 0) {
            MdpJitPlan &plan = eng->jit_plan;
            if (vlds) {  // the wide years' states in LDS: one point per lane, never fused
                plan.vlds = true;
                // points per lane: 1, or 2 (MDP_VLDS_EPL=2: 128 lanes per wave
                // group, each Q read shared by two points)
                const char *ve = eng->opts.get("MDP_VLDS_EPL");
                plan.epl = ve && atoi(ve) == 2 ? 2 : 1;
                plan.kblock = (int)vkb / plan.epl;
                plan.window = 16;
                eng->fused_mode = 0;
                if (const char *sv = eng->opts.get("MDP_VSPLIT")) plan.vsplit = atoi(sv) == 1 ? 1 : atoi(sv) == 2 ? 2 : 4;
            }
            plan.np = eng->np;
            plan.udesc = eng->udesc_d;
            plan.ldQ = eng->ldQ;
            plan.diag = eng->diag;
            if (const char *cv = eng->opts.get("MDP_JIT_SLOTS")) plan.slots = atoi(cv);
            if (const char *wv = eng->opts.get("MDP_JIT_WPE")) plan.wpe = atoi(wv);
            if (const char *xv = eng->opts.get("MDP_JIT_XCD")) plan.xcd = atoi(xv) != 0;
            if (const char *fv2 = eng->opts.get("MDP_JIT_EFAST")) plan.efast = atoi(fv2) != 0;
            if (const char *qx = eng->opts.get("MDP_QROWS_XCD")) eng->qrows_xcd = atoi(qx) != 0;
            if (const char *ev = eng->opts.get("MDP_EPL")) {
                plan.epl = atoi(ev);
                eng->jit_shape_env = true;
            }
            if (const char *wv = eng->opts.get("MDP_JIT_WINDOW")) plan.window = atoi(wv);
            // compile the variant a small grid uses now (the other on demand)
            if (const char *fv = eng->opts.get("MDP_FUSED")) eng->fused_mode = atoi(fv) != 0;
            if (const char *cv = eng->opts.get("MDP_FUSED_COLS")) plan.fused_cols = std::max(1, std::min(4, atoi(cv)));
            if (const char *cv = eng->opts.get("MDP_JIT_HACK")) plan.hack = atoi(cv);
            if (const char *cv = eng->opts.get("MDP_FAST_LOG")) plan.fast_log = atoi(cv) != 0;
            if (const char *cv = eng->opts.get("MDP_JIT_KBLOCK"); cv && !vlds) {
                plan.kblock = atoi(cv) == 512 ? 512 : 256;
                eng->jit_shape_env = true;
            }
            plan.nj = eng->nj;
            plan.nvar = eng->nvar;
            plan.nitems = eng->nitems;
            plan.ncoef = eng->ncoef_d;
            plan.nqi = (uint32_t)eng->qitem.size();
            {   // zs rows compiled into the fused kernel: the longest row of
                // explicit columns at |c| <= 1 (the default grid); a grid
                // with more (|c| > 1) runs k_zrows + k_qrows instead
                size_t kz = 0;
                std::vector<double> large;
                for (uint32_t js = 0; js < eng->nj; ++js) {
                    z_split(eng, js, 1.0, large, nullptr);
                    kz = std::max(kz, large.size());
                }
                plan.kzmax = (uint32_t)std::max<size_t>(8, (kz + 7) & ~(size_t)7);
            }
            plan.qmaxlen = 0;
            for (size_t q = 0; q + 1 < eng->qstart.size(); ++q)
                plan.qmaxlen = std::max(plan.qmaxlen, eng->qstart[q + 1] - eng->qstart[q]);
            auto even = [](size_t v) { return (uint32_t)((v + 1) & ~(size_t)1); };
            if (const char *sv = eng->opts.get("MDP_JIT_SPLIT")) plan.split_forms = atoi(sv) != 0;
            if (const char *sv = eng->opts.get("MDP_JIT_ROT")) plan.rot = atoi(sv) != 0;
            {
                plan.off_it = even((size_t)eng->nj * eng->nvar);
                plan.off_qs = even(plan.off_it + eng->nitems);
                plan.off_qi = even(plan.off_qs + (eng->ncoef_d + 2) / 2);
                plan.off_rq = even(plan.off_qi + (eng->qitem.size() + 1) / 2);
                plan.off_zc = even(plan.off_rq + (eng->ldQ + 1) / 2);
                plan.off_zs = even(plan.off_zc + (size_t)eng->nj * kZTerms);
                const size_t kmax_max = plan.kzmax;
                plan.ct_max = (uint32_t)std::min<size_t>(((plan.off_zs + kmax_max * eng->nj) + 127) & ~(size_t)127,
                                                         kFusedLdsMax / sizeof(double));
                // zero-padded zs image when the largest one fits the fused kernel's LDS
                const size_t kz = std::max<size_t>(8, kmax_max);
                plan.zpad = fused_lds(eng, ((plan.off_zs + kz * eng->nj) + 127) & ~(size_t)127) <= kFusedLdsMax;
            }
            if (chunked && (rc = plan_chunks(eng, chunk_uses, gather, qlimit))) {
                delete eng;
                return rc;
            }
            if (jit_check && ndev == 0 && chunked) {
                const int r = jit_build_chunks(eng);
                if (!r)
                    mdp_set_error(MDP_ENODEV, "no HIP device available (forward kernels compiled; %zu chunks%s; "
                                  "nj %u nitems %u ldQ %zu qglobal %d)", eng->chunks.size(), gather ? ", gathered Q" : "",
                                  plan.nj, plan.nitems, (size_t)plan.ldQ, (int)eng->qglobal);
                delete eng;
                return r ? r : MDP_ENODEV;
            }
            if (jit_check && ndev == 0) {
                const int r0 = jit_build(eng, false), r1 = r0 ? r0 : jit_build(eng, true);
                uint32_t ipr = 0;  // most items of one row
                for (uint32_t js = 0; js + 1 < eng->cj_item0.size(); ++js)
                    ipr = std::max(ipr, eng->cj_item0[js + 1] - eng->cj_item0[js]);
                if (!r1)
                    mdp_set_error(MDP_ENODEV,
                                  "no HIP device available (forward kernels compiled; nj %u nitems %u "
                                  "items/row %u ldQ %zu qitems %u qmaxlen %u kzmax %u qrows slots %u conflicts %u + %u fused LDS %zu)",
                                  plan.nj, plan.nitems, ipr, (size_t)plan.ldQ, plan.nqi, plan.qmaxlen, plan.kzmax,
                                  eng->npl_slots, eng->slot_conflicts, eng->slot_store_conflicts,
                                  fused_lds(eng, ((plan.off_zs + (size_t)plan.kzmax * eng->nj) + 127) & ~(size_t)127));
                delete eng;
                return r1 ? r1 : MDP_ENODEV;
            }
            // compile now the variant the first grid most likely runs (the
            // fused kernel wherever its tables fit: every grid of at most one
            // e block per column takes it), the other on demand (set_grid_dev)
            const bool fused_first = eng->fused_mode == 1 ||
                                     (eng->fused_mode == -1 && !vlds && !eng->qglobal &&
                                      fused_lds(eng, plan.ct_max) <= kFusedLdsMax);
            st_jit0 = st_now();
            const int jrc = chunked ? jit_build_chunks(eng) : jit_build(eng, fused_first);
            st_jit1 = st_now();
            if (jrc == MDP_OK) eng->jit = true;
            else fprintf(stderr, "midaspom: hipRTC specialisation failed, using the %s kernels:\n%s\n",
                         vlds ? "wide" : "generic", eng->jit_log.c_str());
        }
        if (vlds && !eng->jit) {  // no specialised kernel after all: the wide kernels take the problem
            eng->wide = true;
            eng->qglobal = false;
            eng->chunks.clear();
        } else if (vlds) {
            eng->variant = (eng->npmax <= 32 ? 32u : eng->npmax <= 64 ? 64u : 128u) * 100u + eng->deg;
        }
    }
    if (eng->wide) {
        if ((rc = build_wide_plan(eng, p))) {
            delete eng;
            return rc;
        }
        if (jit_check && ndev == 0) {
            delete eng;
            return mdp_set_error(MDP_ENODEV, "no HIP device available (wide path planned)");
        }
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
    const double st_dev0 = st_now();
    for (size_t i = 0; i < ids.size(); ++i) {
        eng->devs[i].device = ids[i];
        rc = init_device(eng, eng->devs[i], p);
        if (rc) {
            mdp_engine_destroy(eng);
            return rc;
        }
    }
    if (st_on)
        fprintf(stderr, "mdp setup (s): plan %.3f jit %.3f plan2 %.3f devices %.3f\n", st_jit0 - st0, st_jit1 - st_jit0,
                st_dev0 - st_jit1, st_now() - st_dev0);
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

int mdp_engine_set_cbound(mdp_engine *eng, double cbound)
{
    if (!eng) return mdp_set_error(MDP_EINVAL, "null argument");
    if (!(cbound >= 0.0) || std::isinf(cbound)) return mdp_set_error(MDP_EINVAL, "cbound %g (want a finite value >= 0)", cbound);
    eng->cbound = cbound;
    return MDP_OK;
}

int mdp_engine_set_layout(mdp_engine *eng, int layout)
{
    if (!eng) return mdp_set_error(MDP_EINVAL, "null argument");
    if (layout != MDP_LAYOUT_EC && layout != MDP_LAYOUT_CE) return mdp_set_error(MDP_EINVAL, "unknown layout %d", layout);
    eng->layout = layout;
    return MDP_OK;
}

int mdp_engine_run(mdp_engine *eng, double *d_out, uint32_t ld_out, void *stream)
{
    if (!eng || !d_out) return mdp_set_error(MDP_EINVAL, "null argument");
    if (eng->devs.size() != 1)
        return mdp_set_error(MDP_EINVAL, "mdp_engine_run needs a single-device engine");
    DevCtx &d = eng->devs[0];
    if (eng->layout == MDP_LAYOUT_CE ? ld_out < d.ne : ld_out < d.nc)
        return mdp_set_error(MDP_EINVAL, "ld_out %u < %s %u", ld_out, eng->layout == MDP_LAYOUT_CE ? "ne" : "nc",
                             eng->layout == MDP_LAYOUT_CE ? d.ne : d.nc);
    // the caller's stream as given: NULL is HIP's null stream (torch's default
    // stream), never the engine's private non-blocking stream
    return run_dev(eng, d, d_out, layout_strides(eng->layout, ld_out), (hipStream_t)stream);
}

int mdp_loglik_grid(mdp_engine *eng, const double *e, uint32_t ne, const double *c, uint32_t nc,
                    double *out)
{
    return mdp_loglik_grid_layout(eng, e, ne, c, nc, MDP_LAYOUT_EC, out);
}

int mdp_loglik_grid_layout(mdp_engine *eng, const double *e, uint32_t ne, const double *c, uint32_t nc, int layout,
                           double *out)
{
    if (!eng || !out || (ne && !e) || (nc && !c)) return mdp_set_error(MDP_EINVAL, "null argument");
    if (layout != MDP_LAYOUT_EC && layout != MDP_LAYOUT_CE) return mdp_set_error(MDP_EINVAL, "unknown layout %d", layout);
    const bool ce = layout == MDP_LAYOUT_CE;
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
        // the layout asked of this call (not the engine's mdp_engine_run
        // layout): the slab [e][c] (ld nc) or [c][e] (ld = the slab's rows)
        if ((rc = run_dev(eng, d, d.out, ce ? OutStrides{1u, rows} : OutStrides{nc, 1u}, d.stream))) return rc;
    }
    for (uint32_t r = 0; r < nd; ++r) {
        DevCtx &d = eng->devs[r];
        const uint32_t rows = r1[r] - r0[r];
        HIP_TRY(hipSetDevice(d.device));
        if (rows && !ce)
            HIP_TRY(hipMemcpyAsync(out + (size_t)r0[r] * nc, d.out, (size_t)rows * nc * sizeof(double),
                                   hipMemcpyDeviceToHost, d.stream));
        else if (rows && nc)  // the slab's columns into out[c][e] at e offset r0
            HIP_TRY(hipMemcpy2DAsync(out + r0[r], (size_t)ne * sizeof(double), d.out, (size_t)rows * sizeof(double),
                                     (size_t)rows * sizeof(double), nc, hipMemcpyDeviceToHost, d.stream));
    }
    for (uint32_t r = 0; r < nd; ++r) {
        HIP_TRY(hipSetDevice(eng->devs[r].device));
        HIP_TRY(hipStreamSynchronize(eng->devs[r].stream));
    }
    for (uint32_t r = nd; r-- > 0;)  // device 0 last: its means are reported
        if ((rc = collect_times(eng, eng->devs[r]))) return rc;
    return MDP_OK;
}

int mdp_engine_diag_report(mdp_engine *eng, char *buf, size_t len)
{
    if (!eng || !buf || !len) return mdp_set_error(MDP_EINVAL, "null argument");
    buf[0] = 0;
    if (!eng->diag || eng->devs.empty()) return 0;
    DevCtx &d = eng->devs[0];
    HIP_TRY(hipSetDevice(d.device));
    HIP_TRY(hipDeviceSynchronize());
    const char *names[3] = {"k_zpv", "k_coefs", "k_forward_lds"};
    int slots[3] = {3, 5, 3};
    if (eng->jit) {  // direct path: k_qrows and the hipRTC forward kernel
        names[1] = "k_qrows";
        names[2] = "k_forward(jit)";
        slots[0] = 0;
        slots[1] = 6;  // k_qrows stamps slots 4 and 5 inside phase 1
        slots[2] = d.fused ? 6 : 4;
    }
    size_t used = 0;
    for (int k = 0; k < 3; ++k) {
        if (!d.stamps[k] || !d.nst[k] || !slots[k]) continue;
        std::vector<unsigned long long> h(d.nst[k] * kStampSlots);
        HIP_TRY(hipMemcpy(h.data(), d.stamps[k], h.size() * sizeof(unsigned long long),
                          hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull, t1 = 0, rs0 = ~0ull, rs1 = 0, re1 = 0;
        double rdur = 0.0;
        std::vector<double> mean(slots[k], 0.0);
        size_t nb = 0;
        for (size_t b = 0; b < d.nst[k]; ++b) {
            const unsigned long long *st = &h[b * kStampSlots];
            const int last = ((k == 2 && d.fused) || k == 1) && eng->jit ? 3 : slots[k] - 1;
            if (!st[0] || !st[last] || st[last] < st[0]) continue;
            ++nb;
            rs0 = std::min(rs0, st[6]);
            rs1 = std::max(rs1, st[6]);
            re1 = std::max(re1, st[7]);
            rdur += (double)(st[7] - st[6]);
            t0 = std::min(t0, st[0]);
            t1 = std::max(t1, st[last]);
            // the fused forward kernel stamps slots 4 and 5 between 0 and 1
            const bool fz = ((k == 2 && eng->devs[0].fused) || k == 1) && eng->jit && slots[k] == 6;
            static const int seq_plain[6] = {0, 1, 2, 3, 4, 5}, seq_fused[6] = {0, 4, 5, 1, 2, 3};
            const int *seq = fz ? seq_fused : seq_plain;
            for (int q = 1; q < slots[k]; ++q) mean[q] += (double)(st[seq[q]] - st[seq[q - 1]]);
        }
        int w = snprintf(buf + used, len - used,
                         "%s: blocks=%zu wall_us=%.2f last_start_us=%.2f mean_block_us=%.2f cycles:",
                         names[k], nb, nb ? (re1 - rs0) * 0.01 : 0.0, nb ? (rs1 - rs0) * 0.01 : 0.0,
                         nb ? rdur / nb * 0.01 : 0.0);
        if (w > 0) used = std::min(len - 1, used + (size_t)w);
        for (int q = 1; q < slots[k]; ++q) {
            w = snprintf(buf + used, len - used, " ph%d=%.0f", q, nb ? mean[q] / nb : 0.0);
            if (w > 0) used = std::min(len - 1, used + (size_t)w);
        }
        {   // block start / end spread (wall clock): percentiles, and the latest start per XCD
            std::vector<double> st0, en;
            double xmax[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            for (size_t b = 0; b < d.nst[k]; ++b) {
                const unsigned long long *st = &h[b * kStampSlots];
                if (!st[6] || !st[7] || st[7] < st[6] || st[6] < rs0) continue;
                st0.push_back((st[6] - rs0) * 0.01);
                en.push_back((st[7] - rs0) * 0.01);
                xmax[b % 8] = std::max(xmax[b % 8], (st[6] - rs0) * 0.01);
            }
            if (!st0.empty()) {
                std::sort(st0.begin(), st0.end());
                std::sort(en.begin(), en.end());
                auto pc = [](const std::vector<double> &v, double f) { return v[(size_t)(f * (v.size() - 1))]; };
                w = snprintf(buf + used, len - used,
                             " start_us p10=%.2f p50=%.2f p90=%.2f p99=%.2f end_us p1=%.2f p50=%.2f max=%.2f "
                             "xcd_last_start_us=%.2f,%.2f,%.2f,%.2f,%.2f,%.2f,%.2f,%.2f",
                             pc(st0, 0.1), pc(st0, 0.5), pc(st0, 0.9), pc(st0, 0.99), pc(en, 0.01), pc(en, 0.5),
                             en.back(), xmax[0], xmax[1], xmax[2], xmax[3], xmax[4], xmax[5], xmax[6], xmax[7]);
                if (w > 0) used = std::min(len - 1, used + (size_t)w);
            }
        }
        if (k == 2 && nb && !eng->jit) {  // forward: cycles summed over run ops / general ops (wave 0)
            double cr = 0, cg = 0;
            for (size_t b = 0; b < d.nst[k]; ++b) {
                const unsigned long long *st = &h[b * kStampSlots];
                if (!st[0] || !st[2]) continue;
                cr += (double)st[3];
                cg += (double)st[4];
            }
            w = snprintf(buf + used, len - used, " run_ops=%.0f general_ops=%.0f", cr / nb, cg / nb);
            if (w > 0) used = std::min(len - 1, used + (size_t)w);
        }
        w = snprintf(buf + used, len - used, "\n");
        if (w > 0) used = std::min(len - 1, used + (size_t)w);
        HIP_TRY(hipMemset(d.stamps[k], 0, h.size() * sizeof(unsigned long long)));
    }
    return (int)used;
}

int mdp_engine_set_profiling(mdp_engine *eng, int enable)
{
    if (!eng) return mdp_set_error(MDP_EINVAL, "null engine");
    eng->profiling = enable;
    return MDP_OK;
}

int mdp_engine_time_kernels(mdp_engine *eng, double *d_out, uint32_t ld_out, void *stream, int reps,
                            double *ms, int max_k)
{
    if (!eng || !d_out || !ms || reps < 1) return mdp_set_error(MDP_EINVAL, "bad argument");
    if (eng->devs.size() != 1)
        return mdp_set_error(MDP_EINVAL, "mdp_engine_time_kernels needs a single-device engine");
    DevCtx &d = eng->devs[0];
    if (eng->layout == MDP_LAYOUT_CE ? ld_out < d.ne : ld_out < d.nc)
        return mdp_set_error(MDP_EINVAL, "ld_out %u < %s %u", ld_out, eng->layout == MDP_LAYOUT_CE ? "ne" : "nc",
                             eng->layout == MDP_LAYOUT_CE ? d.ne : d.nc);
    double t[3];
    const int saved = eng->profiling;
    eng->profiling = 0;
    int rc = time_kernels(eng, d, d_out, layout_strides(eng->layout, ld_out), (hipStream_t)stream, reps, t);
    eng->profiling = saved;
    if (rc) return rc;
    const int k = std::min(max_k, 3);
    for (int i = 0; i < k; ++i) ms[i] = t[i];
    return k;
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

const char *mdp_engine_kernel_name(const mdp_engine *eng, int k)
{
    if (!eng || k < 0 || k >= 3) return "";
    if (eng->wide && eng->hs) return k == 0 && eng->nitems ? "k_zrows" : k == 1 && eng->nitems ? "k_witems" : k == 2 ? "k_fwd_hs" : "";
    if (eng->wide) return k < 2 && !eng->nitems ? "" : k == 2 && eng->mmt ? "k_fwd_mmt" : k == 2 && eng->mma ? "k_fwd_mma" : kKernelNames[2][k];
    if (eng->jit && eng->qglobal)  // Q rows built in HBM, then the hipRTC forward kernel
        return k < 2 && !eng->nitems ? "" : k == 2 ? "k_forward" : kKernelNames[2][k];
    // direct path: Z rows inside k_qrows (slot 0 idle); fused: one kernel
    if (eng->jit && (k == 0 || (k == 1 && (eng->devs.empty() || eng->devs[0].fused)))) return "";
    return kKernelNames[eng->jit ? 1 : 0][k];
}

int mdp_log_check(const double *x, double *y, size_t n)
{
    if ((n && (!x || !y))) return mdp_set_error(MDP_EINVAL, "null argument");
    if (!n) return MDP_OK;
    std::vector<char> code;
    std::string log;
    if (mdp_jit_compile(mdp_jit_log_source(), code, log) != 0)
        return mdp_set_error(MDP_EHIP, "hipRTC compilation of mdp_log failed: %s", log.c_str());
    hipModule_t mod = nullptr;
    hipFunction_t fn;
    double *dx = nullptr, *dy = nullptr;
    int rc = MDP_OK;
    auto fail = [&](hipError_t e, const char *what) {
        rc = mdp_set_error(MDP_EHIP, "%s failed: %s", what, hipGetErrorString(e));
    };
    hipError_t e;
    if ((e = hipModuleLoadData(&mod, code.data())) != hipSuccess) fail(e, "hipModuleLoadData");
    else if ((e = hipModuleGetFunction(&fn, mod, "mdp_log_apply")) != hipSuccess) fail(e, "hipModuleGetFunction");
    else if ((e = hipMalloc((void **)&dx, n * sizeof(double))) != hipSuccess) fail(e, "hipMalloc");
    else if ((e = hipMalloc((void **)&dy, n * sizeof(double))) != hipSuccess) fail(e, "hipMalloc");
    else if ((e = hipMemcpy(dx, x, n * sizeof(double), hipMemcpyHostToDevice)) != hipSuccess) fail(e, "hipMemcpy");
    else {
        unsigned long long nn = n;
        void *args[] = {(void *)&dx, (void *)&dy, (void *)&nn};
        const uint32_t nb = (uint32_t)((n + kBlock - 1) / kBlock);
        if ((e = hipModuleLaunchKernel(fn, nb, 1, 1, kBlock, 1, 1, 0, nullptr, args, nullptr)) != hipSuccess)
            fail(e, "hipModuleLaunchKernel");
        else if ((e = hipMemcpy(y, dy, n * sizeof(double), hipMemcpyDeviceToHost)) != hipSuccess) fail(e, "hipMemcpy");
    }
    (void)hipFree(dx);
    (void)hipFree(dy);
    if (mod) (void)hipModuleUnload(mod);
    return rc;
}

int mdp_engine_launched(const mdp_engine *eng, char *buf, size_t len)
{
    if (!eng || !buf || !len) return mdp_set_error(MDP_EINVAL, "null argument");
    std::string all;
    {
        std::lock_guard<std::mutex> lk(eng->launched_mu);
        for (const std::string &k : eng->launched) all += (all.empty() ? "" : " ") + k;
    }
    snprintf(buf, len, "%s", all.c_str());
    return (int)all.size();
}

int mdp_engine_get_info(const mdp_engine *eng, mdp_engine_info *info)
{
    if (!eng || !info) return mdp_set_error(MDP_EINVAL, "null argument");
    info->n_devices = (int)eng->devs.size();
    info->npairs = eng->npairs;
    info->nuses = eng->nuses;
    info->ncoef = eng->ncoef;
    info->npmax = eng->npmax;
    info->variant = eng->variant + (eng->jit ? 10000u : 0u);
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
    if (eng->jit) per_pt = eng->jit_flops_pt;  // the generated code's own count
    if (eng->wide) per_pt = eng->hs ? eng->hs_flops_pt : eng->mmt ? eng->mmt_flops_pt : eng->wide_flops_pt;
    if (flop_impl) *flop_impl = per_pt * pts;
    // SURVEY.md §8(d) F_alg (dense-in-j formulation)
    double fwd = 0;
    for (uint32_t t = 1; t < eng->tmax; ++t) fwd += (double)eng->np[t - 1] * eng->np[t];
    const double falg = 2.0 * eng->n * eng->nstates + (double)eng->nvar * eng->nstates * eng->nextid +
                        2.0 * eng->nstates * eng->npairs + 2.0 * eng->np[0] * fwd;
    if (flop_survey) *flop_survey = falg * pts;
    // compulsory bytes of k_forward: its coefficient stream once per c, the
    // e values, the output
    if (bytes_min)
        *bytes_min = 8.0 * ((double)nc * (eng->jit || eng->wide ? eng->ldQ : ldR_of(eng)) + (double)ne + pts);
    return MDP_OK;
}


int mdp_engine_work_fact(const mdp_engine *eng, uint64_t ne, uint64_t nc, mdp_work *w)
{
    if (!eng || !w) return mdp_set_error(MDP_EINVAL, "null argument");
    *w = mdp_work{};
    // per c value (the direct plan's tables; zero on the generic path, which
    // has none): Z rows, var-column pressures, item factors, Q sums
    double cmax = eng->devs.empty() ? 1.0 : eng->devs[0].zs_cmax;
    if (!(cmax >= 0.0)) cmax = 1.0;  // no grid yet: the default [0, 1]
    std::vector<double> large;
    double coef[kZTerms];
    for (uint32_t js = 0; js < eng->nj; ++js) {
        z_split(eng, js, cmax, large, coef);
        // fma(-c, s, 1) and one multiply per explicit column; the small
        // columns' series: kZTerms FMAs, a multiply, the exp (counted 1)
        w->z_c += 3.0 * (double)large.size() + (coef[0] != 0.0 ? 2.0 * kZTerms + 2.0 : 0.0);
        w->pc_c += (double)eng->nvar;  // pC = c S[j][b] per var column
    }
    const uint32_t vmask = eng->nvar >= 32 ? ~0u : (1u << eng->nvar) - 1u;
    for (uint32_t i = 0; i < eng->nitems; ++i) {
        const uint32_t j = eng->cj_bits[eng->itemRow[i]], B = eng->itemB[i];
        const uint32_t free = (uint32_t)__builtin_popcount(~j & vmask);
        // 1 - pC where B_b = 0, one multiply per free column (the last one by Z)
        w->item_c += (double)__builtin_popcount(~B & ~j & vmask) + (double)free;
    }
    for (size_t q = 0; q + 1 < eng->qstart.size(); ++q) {
        const uint32_t len = eng->qstart[q + 1] - eng->qstart[q];
        if (len > 1) w->q_c += (double)(len - 1);
    }
    // per grid point: the weight table, every use's (nX+1)-term dot product
    // and its multiply-add into the state vector, the final prior sum
    std::vector<int> wmax(kMaxDeg + 1, -1);
    const std::vector<uint32_t> &ud = eng->udesc_d.empty() ? eng->udesc : eng->udesc_d;
    std::set<uint32_t> distinct;  // one descriptor = one transition value P(e, c)
    for (uint32_t d : ud) {
        const uint32_t nX = (d >> kOffBits) & 31u, nA = d >> 27;
        wmax[nA] = std::max(wmax[nA], (int)nX);
        w->use_pt += 2.0 * nX + 3.0;
        if (distinct.insert(d).second) w->use_pt_min += 2.0 * nX + 1.0;  // the dot product, once
    }
    // the state updates v'[l] = sum_k v[k] P[k][l]: npc (2 npp - 1) per year
    for (uint32_t t = 1; t < eng->tmax; ++t) w->use_pt_min += (double)eng->np[t] * (2.0 * eng->np[t - 1] - 1.0);
    w->weight_pt = 2.0 * eng->maxA;
    for (int a = 0; a <= kMaxDeg; ++a)
        if (wmax[a] >= 0) w->weight_pt += (double)(wmax[a] + 1);
    w->final_pt = 2.0 * eng->np[eng->tmax - 1] - 1.0;
    const double per_c = w->z_c + w->pc_c + w->item_c + w->q_c;
    const double per_pt = w->weight_pt + w->use_pt + w->final_pt;
    w->flop = (double)nc * per_c + (double)ne * (double)nc * per_pt;
    w->flop_min_direct = (double)nc * per_c + (double)ne * (double)nc * (w->weight_pt + w->use_pt_min + w->final_pt);
    // the ratio forms (ABI 8): per form from the plan, then the mean over the
    // current grid's e rows (half s-form before a grid is set)
    MdpJitPlan pl;
    pl.np = eng->np;
    pl.udesc = ud;
    const MdpRatioWork rw = mdp_jit_ratio_work(pl);
    double ns = 0.0, nall = 0.0;
    for (const DevCtx &d : eng->devs) {
        ns += d.ne_sform;
        nall += d.ne;
    }
    const double fs = nall > 0.0 ? ns / nall : 0.5;
    w->setup_pt = fs * rw.setup_s + (1.0 - fs) * rw.setup_t;
    w->use_pt_ratio = fs * rw.use_s + (1.0 - fs) * rw.use_t;
    w->final_pt_ratio = rw.final_pt;
    w->pt_min = w->setup_pt + w->use_pt_ratio + w->final_pt_ratio;
    w->flop_min = (double)nc * per_c + (double)ne * (double)nc * w->pt_min;
    return MDP_OK;
}

}  // extern "C"
