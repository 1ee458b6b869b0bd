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
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "mdp_internal.h"

namespace {

constexpr int kScnBlock = 1024;       // 16 waves: four per SIMD
constexpr bool kPingPong = kScnBlock <= 768;  // register double-buffering (needs > 128 VGPRs)
constexpr bool kDppFactors = true;  // hi factors by DPP row broadcast (fma_rowbcast) instead of LDS broadcasts
constexpr int kE = 32;                 // e values per workgroup (lanes mod 32)
constexpr int kWaves = kScnBlock / 64;
constexpr uint32_t kMaxN = 8;          // k_scn: 2 x 2^8 x 32 state values + factor tables in LDS
constexpr uint32_t kBigMaxN = 16;      // k_scn_big: state vectors in HBM
constexpr int kBigBlock = 256;
constexpr size_t kBigScratch = 1ull << 30;  // k_scn_big state-vector scratch per launch (bytes)
constexpr int kRowBlock = 256;              // k_scn_row: one grid point per workgroup
constexpr uint32_t kRowMaxN = 12;           // k_scn_row: 2 x 2^n states + 3 n x 256 per-lane values in LDS

#define SCN_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return mdp_set_error(MDP_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                                 __FILE__, __LINE__);                                        \
    } while (0)

struct ScnArgs {
    uint32_t n, ns, ne, nc, nK, nd;
    int years;          // tdis (mode 0) or ts (mode 1)
    int loss;           // 0 die-off, 1 habitat loss
    int mode;           // 0: y0 = prior w, store v = P^tdis w;  1: y0 = v, L = 1^T PK^ts v
    uint32_t nsched;    // hi-row slots per wave in jsched
    uint32_t btot;      // doubles of the hi factor table
};

__host__ __device__ constexpr int pow3(int x)
{
    int r = 1;
    for (; x > 0; --x) r *= 3;
    return r;
}
__host__ __device__ constexpr int popc_c(int x)
{
    int c = 0;
    for (; x; x >>= 1) c += x & 1;
    return c;
}
// offset of lo row jl in a hi row's lo factor block: rows ascending, row jl
// holding its 2^(NL - |jl|) supersets bl ascending
__host__ __device__ constexpr int aoff(int NL, int jl)
{
    int o = 0;
    for (int i = 0; i < jl; ++i) o += 1 << (NL - popc_c(i));
    return o;
}
// rank of superset bl among the supersets of jl (ascending)
__host__ __device__ constexpr int sup_rank(int NL, int jl, int bl)
{
    // deposit order of the free bits is ascending bit position, so the rank is
    // the free bits of bl read from high to low (the highest free bit is the
    // most significant)
    int r = 0;
    for (int b = NL - 1; b >= 0; --b)
        if (!((jl >> b) & 1)) r = 2 * r + ((bl >> b) & 1);
    return r;
}

// acc + (lane K of this lane's row of 16)'s f * x: v_fmac_f64 with a DPP
// row_newbcast source (gfx950), so a wave-half-uniform factor reaches every
// lane of its row without a broadcast LDS read or an extra move.  A DPP
// source must not be written by a VALU instruction in the two before it; f is
// always a value just loaded from LDS (no VALU write), and the compiled k_scn
// was checked for such a pair (none).  All lanes are active
// where it is used (wave-uniform loops).
template <int K>
__device__ __forceinline__ double fma_rowbcast(double f, double x, double acc)
{
    asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
        : "+v"(acc)
        : "v"(f), "v"(x), "i"(K));
    return acc;
}

// lanes 0-31: a[lane] + a[lane + 32]; lanes 32-63: b[lane - 32] + b[lane]
// (one v_permlane32_swap per 32-bit word, no copies: both outputs are used)
__device__ __forceinline__ double pair_sum(double a, double b)
{
    const auto l2 = __builtin_amdgcn_permlane32_swap(__double2loint(a), __double2loint(b), false, false);
    const auto h2 = __builtin_amdgcn_permlane32_swap(__double2hiint(a), __double2hiint(b), false, false);
    return __hiloint2double(h2[0], l2[0]) + __hiloint2double(h2[1], l2[1]);
}

__device__ __forceinline__ uint32_t deposit(uint32_t r, uint32_t mask)  // r's bits into mask, ascending
{
    uint32_t b = 0;
    for (uint32_t t = 0; mask; ++t) {
        const uint32_t low = mask & (0u - mask);
        if ((r >> t) & 1u) b |= low;
        mask ^= low;
    }
    return b;
}

// One workgroup = one (c, K, dsrc) point (mode 1) or one c (mode 0) x kE e
// values; lanes run over e.  A state s = (h << NL) | l splits into NH "hi"
// patches (patches 0..NH-1, the top bits) and NL "lo" patches.  The
// colonisation factor of row j and superset b factorises as
//     Pc[j][b] = B_j(b_hi) * A_j(b_lo),
// each the reference's product over its patches k not in j, ascending k
// (dieoff.c:66-83, loss.c:86-105), so
//     (Pc y)[j] = sum_{bh >= jh} B_j(bh) * sum_{bl >= jl} A_j(bl) y[bh][bl].
// A wave owns one hi row jh at a time (an LPT schedule over the waves); its
// two 32-lane halves split the supersets bh.  Per (jh, bh) the 2^NL values
// y[bh][.] are loaded once into registers and serve all 3^NL terms of the
// 2^NL rows (jh, .) -- the register blocking that keeps LDS traffic under
// the FP64 rate -- with the 3^NL lo factors of jh held in registers across
// its supersets.  Extinction (Pe, a tensor product over patches: per patch
// y[s | m] = E y[s] + (1 - E) y[s | m]) is applied to the lo patches in
// registers at the end of each hi row and to the hi patches in a second
// phase where each thread holds the 2^NH hi states of one (lo, e).
template <int NL, int NH>
__global__ __launch_bounds__(kScnBlock) void k_scn(ScnArgs a, const double *__restrict__ S,
                                                    const double *__restrict__ y0src, const double *__restrict__ ev,
                                                    const double *__restrict__ cv, const double *__restrict__ Kv,
                                                    const double *__restrict__ srcv, const uint32_t *__restrict__ boff,
                                                    const uint32_t *__restrict__ jsched, double *__restrict__ out)
{
    constexpr int NLO = 1 << NL, NHI = 1 << NH, NS = NLO * NHI, NA = pow3(NL), NAP = (NA + 1) & ~1, N = NL + NH;
    constexpr int LS = NHI * kE + 2;  // lo row stride (doubles); see below
    // state (h, l) of lane e at [l LS + h kE + e]: lo-major with a stride
    // that no ds_read2 / ds_read2st64 offset pair can express, so the 2^NL
    // lo states of one hi state load as separate ds_read_b64 (a merged read2
    // costs twice the LDS cycles per byte, MI355X_MICROARCH.md LDS table)
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double *y = lds;                      // [NLO][LS] current states
    double *yb = y + NLO * LS;            // [NLO][LS] after colonisation
    double *At = yb + NLO * LS;           // [NHI][NAP] lo factors
    double *Bt = At + NHI * NAP;          // per hi row jh: [2^(NH-|jh|)][NLO] hi factors
    double *pc = yb;                      // [NS][N] colonisation pressures (before yb is used)
    __shared__ double Es[kE];
    const uint32_t tid = threadIdx.x;
    const uint32_t nchunk = (a.ne + kE - 1) / kE;
    const uint32_t pt = blockIdx.x / nchunk, chunk = blockIdx.x % nchunk, e0 = chunk * kE;
    const uint32_t id = a.mode ? pt % a.nd : 0u, iK = a.mode ? (pt / a.nd) % a.nK : 0u;
    const uint32_t ic = a.mode ? pt / (a.nd * a.nK) : pt;
    const double c = cv[ic], K = a.mode ? Kv[iK] : 1.0;
    const double *src = a.mode && a.loss ? srcv + (size_t)id * N : nullptr;
    const double Kpc = a.mode && !a.loss ? K : 1.0;
    // initial states: every load of the thread issued first (unconditionally,
    // to a valid address), so their global round trip overlaps the table
    // build; stored to y after it
    constexpr int kIS = (NS * kE + kScnBlock - 1) / kScnBlock;
    double t0[kIS];
#pragma unroll
    for (int u = 0; u < kIS; ++u) {
        const uint32_t i = tid + u * kScnBlock, x = (i / kE) % NS, le = i % kE;
        const uint32_t st = ((x % NHI) << NL) | (x / NHI);
        const bool ok = !a.mode || e0 + le < a.ne;
        const size_t idx = a.mode ? ((size_t)ic * NS + st) * a.ne + e0 + le : st;
        const double v = y0src[ok ? idx : 0];
        t0[u] = ok ? v : 0.0;
    }
    // hi-row offsets of the factor table, for the flat build below
    __shared__ uint32_t boffs[NHI];
    if (tid < (uint32_t)NHI) boffs[tid] = boff[tid];
    // pC for every (j, k), k not in j: dieoff.c:78 (c S) K, loss.c:98 c (S + src Ks)
    {  // every S (and source) load of the thread in flight before the first store
        constexpr int kPC = (NS * N + kScnBlock - 1) / kScnBlock;
        double sv[kPC], sr[kPC];
#pragma unroll
        for (int u = 0; u < kPC; ++u) {
            const uint32_t i = tid + u * kScnBlock, ii = i < (uint32_t)(NS * N) ? i : 0u;
            sv[u] = S[ii];
            sr[u] = src ? src[ii % N] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kPC; ++u) {
            const uint32_t i = tid + u * kScnBlock, j = i / N, k = i - j * N;
            double v = 0.0;
            if (!((j >> (N - 1 - k)) & 1u)) {
                v = src ? c * (sv[u] + sr[u] * K) : c * sv[u] * Kpc;
                v = v > 1.0 ? 1.0 : v;
            }
            if (i < (uint32_t)(NS * N)) pc[i] = v;
        }
    }
    if (tid < (uint32_t)kE) {
        const double x = e0 + tid < a.ne ? ev[e0 + tid] : 0.0;
        const double E = a.mode && !a.loss ? x / K : x;  // dieoff.c:56-57 E = e/K; loss.c:57 E = e
        Es[tid] = E > 1.0 ? 1.0 : E;
    }
    __syncthreads();
    // lo factors A_j(bl): patches NH..N-1 (bits NL-1..0), ascending patch
    for (uint32_t i = tid; i < (uint32_t)(NHI * NAP); i += kScnBlock) {
        const uint32_t jh = i / NAP;
        uint32_t q = i - jh * NAP, jl = 0;
        if (q >= (uint32_t)NA) {
            At[i] = 0.0;  // pad
            continue;
        }
        while (q >= (1u << (NL - __popc(jl)))) q -= 1u << (NL - __popc(jl++));
        const uint32_t bl = jl | deposit(q, ~jl & (NLO - 1)), j = (jh << NL) | jl;
        double r = 1.0;
        for (int k = NH; k < N; ++k) {
            const uint32_t bit = 1u << (N - 1 - k);
            if (jl & bit) continue;
            const double p = pc[j * N + k];
            r *= (bl & bit) ? p : 1.0 - p;
        }
        At[i] = r;
    }
    // hi factors B_j(bh): patches 0..NH-1, ascending; [jh][rank of bh][jl].
    // One flat pass over the table (entry t belongs to the last hi row jh
    // with boff[jh] <= t: a binary search over the staged offsets).  The
    // earlier loop over the 2^NH hi rows (a global offset load and a short
    // partial pass each) plus the initial-state round trip after it made the
    // per-workgroup fixed cost 32 ms of config 4's 241 ms; now 10.6 ms
    for (uint32_t t = tid; t < a.btot; t += kScnBlock) {
        uint32_t jh = 0;
#pragma unroll
        for (uint32_t st = NHI / 2; st > 0; st >>= 1)
            if (boffs[jh + st] <= t) jh += st;
        const uint32_t i = t - boffs[jh], fr = ~jh & (NHI - 1);
        const uint32_t r = i / NLO, jl = i % NLO, bh = jh | deposit(r, fr), j = (jh << NL) | jl;
        double v = 1.0;
        for (int k = 0; k < NH; ++k) {
            const uint32_t bit = 1u << (NH - 1 - k);
            if (jh & bit) continue;
            const double p = pc[j * N + k];
            v *= (bh & bit) ? p : 1.0 - p;
        }
        Bt[t] = v;
    }
    if (tid < (uint32_t)NLO) Bt[a.btot + tid] = 0.0;  // zero block (upper half, no free hi bit)
    // initial states: stored into y once the tables are built (loaded first)
#pragma unroll
    for (int u = 0; u < kIS; ++u) {
        const uint32_t i = tid + u * kScnBlock, x = i / kE, le = i % kE;
        if (i < (uint32_t)(NS * kE)) y[(x / NHI) * LS + (x % NHI) * kE + le] = t0[u];
    }
    __syncthreads();
    const uint32_t w = tid / 64, g = (tid >> 5) & 1u, le = tid & 31u;
    const double E = Es[le], E1 = 1.0 - E;
    for (int t = 0; t < a.years; ++t) {
        // colonisation: rows (jh, .) of this wave's hi rows, into yb
        for (uint32_t slot = 0; slot < a.nsched; ++slot) {
            // wave-uniform (readfirstlane): the row's loop bounds, free-patch
            // masks and superset walk stay in scalar registers
            const uint32_t jh = __builtin_amdgcn_readfirstlane(jsched[w * a.nsched + slot]);
            if (jh >= (uint32_t)NHI) break;  // wave-uniform
            const uint32_t fr = ~jh & (NHI - 1), f = __popc(fr);
            const uint32_t top = f ? 1u << (31 - __clz(fr)) : 0u, frp = fr & ~top;
            const uint32_t units = f ? 1u << (f - 1) : 1u;
            double A[NA];
            {
                const double2 *ap = (const double2 *)(At + jh * NAP);
#pragma unroll
                for (int q = 0; q < NA / 2; ++q) {
                    const double2 t2 = ap[q];
                    A[2 * q] = t2.x;
                    A[2 * q + 1] = t2.y;
                }
                if (NA & 1) A[NA - 1] = At[jh * NAP + NA - 1];
            }
            // the upper half takes the supersets with the top free bit; with
            // no free bit it reads the zero block past the table (acc = 0)
            const double *bt = g ? (f ? Bt + boff[jh] + (size_t)units * NLO : Bt + a.btot) : Bt + boff[jh];
            double acc[NLO];
#pragma unroll
            for (int l = 0; l < NLO; ++l) acc[l] = 0.0;
            // superset bh = jh | sub | (upper half ? top : 0): the bits are
            // disjoint, so its states sit at yrow + sub kE (sub wave-uniform)
            const double *yrow = y + (jh | (g ? top : 0u)) * kE + le;
            auto load = [&](uint32_t it, uint32_t sub, double (&yc)[NLO], double (&bv)[NLO]) {
#pragma unroll
                for (int l = 0; l < NLO; ++l) yc[l] = yrow[l * LS + sub * kE];
                const double2 *bp = (const double2 *)(bt + it * NLO);
#pragma unroll
                for (int l = 0; l < NLO / 2; ++l) {
                    const double2 t2 = bp[l];
                    bv[2 * l] = t2.x;
                    bv[2 * l + 1] = t2.y;
                }
            };
            auto accumulate = [&](const double (&yc)[NLO], const double (&bv)[NLO]) {
#pragma unroll
                for (int jl = 0; jl < NLO; ++jl) {
                    double in = 0.0;
#pragma unroll
                    for (int bl = 0; bl < NLO; ++bl)
                        if ((bl & jl) == jl) in = fma(A[aoff(NL, jl) + sup_rank(NL, jl, bl)], yc[bl], in);
                    acc[jl] = fma(bv[jl], in, acc[jl]);
                }
            };
            // the same sums with the hi factors spread over the lanes of each
            // row of 16 (lane k holds factor k of its half's superset): one
            // lane-distinct ds_read_b64 per superset instead of NLO / 2
            // broadcast ds_read_b128 -- half the colonisation phase's LDS
            // cycles -- and the same FMAs, so the same bits
            auto accumulate_dpp = [&](const double (&yc)[NLO], double bvr) {
                double in[NLO];
#pragma unroll
                for (int jl = 0; jl < NLO; ++jl) {
                    in[jl] = 0.0;
#pragma unroll
                    for (int bl = 0; bl < NLO; ++bl)
                        if ((bl & jl) == jl) in[jl] = fma(A[aoff(NL, jl) + sup_rank(NL, jl, bl)], yc[bl], in[jl]);
                }
                static_assert(NLO <= 8, "hi factors of a superset fit a row of 16 lanes");
                acc[0] = fma_rowbcast<0>(bvr, in[0], acc[0]);
                if constexpr (NLO > 1) acc[1] = fma_rowbcast<1>(bvr, in[1], acc[1]);
                if constexpr (NLO > 2) {
                    acc[2] = fma_rowbcast<2>(bvr, in[2], acc[2]);
                    acc[3] = fma_rowbcast<3>(bvr, in[3], acc[3]);
                }
                if constexpr (NLO > 4) {
                    acc[4] = fma_rowbcast<4>(bvr, in[4], acc[4]);
                    acc[5] = fma_rowbcast<5>(bvr, in[5], acc[5]);
                    acc[6] = fma_rowbcast<6>(bvr, in[6], acc[6]);
                    acc[7] = fma_rowbcast<7>(bvr, in[7], acc[7]);
                }
            };
            uint32_t sub = 0;
            if (!kPingPong) {
                // the next superset's states load under this one's FMAs (its
                // hi factors are first needed at the end of each row's chain,
                // so they load in place)
                double yn[NLO];
#pragma unroll
                for (int l = 0; l < NLO; ++l) yn[l] = yrow[l * LS];
                for (uint32_t it = 0; it < units; ++it) {
                    double ya[NLO];
#pragma unroll
                    for (int l = 0; l < NLO; ++l) ya[l] = yn[l];
                    const uint32_t sn = (sub - frp) & frp;  // wraps to 0 after the last
#pragma unroll
                    for (int l = 0; l < NLO; ++l) yn[l] = yrow[l * LS + sn * kE];
                    if (kDppFactors) {
                        accumulate_dpp(ya, bt[it * NLO + (tid & (NLO - 1))]);
                    } else {
                        double ba[NLO];
                        const double2 *bp = (const double2 *)(bt + it * NLO);
#pragma unroll
                        for (int l = 0; l < NLO / 2; ++l) {
                            const double2 t2 = bp[l];
                            ba[2 * l] = t2.x;
                            ba[2 * l + 1] = t2.y;
                        }
                        accumulate(ya, ba);
                    }
                    sub = sn;
                }
            } else {
            // supersets in pairs, ping-pong register buffers: the next
            // superset's states and factors load under this one's FMAs
            double ya[NLO], ba[NLO], yb2[NLO], bb[NLO];
            load(0, 0, ya, ba);
            if (units == 1) {
                accumulate(ya, ba);
            } else {  // units even; the last pair's look-ahead reloads it (in range)
                for (uint32_t it = 0; it < units; it += 2) {
                    const uint32_t s1 = (sub - frp) & frp;
                    load(it + 1, s1, yb2, bb);
                    accumulate(ya, ba);
                    const bool more = it + 2 < units;
                    const uint32_t s2 = more ? (s1 - frp) & frp : s1;
                    load(more ? it + 2 : it + 1, s2, ya, ba);
                    accumulate(yb2, bb);
                    sub = s2;
                    // keep each buffer's loads ahead of the other buffer's FMAs
                    // (the default schedule interleaves them and waits early)
                    __builtin_amdgcn_sched_group_barrier(0x100, 3 * NLO / 2, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, NA + NLO + 8, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 3 * NLO / 2, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, NA + NLO + 8, 0);
                }
            }
            }
            // extinction on the lo patches, ascending patch -- linear, so it
            // is applied to each half's partial sums before they are combined
#pragma unroll
            for (int k = NH; k < N; ++k) {
                const int m = 1 << (N - 1 - k);
#pragma unroll
                for (int l = 0; l < NLO; ++l)
                    if (l & m) acc[l] = E * acc[l ^ m] + E1 * acc[l];
            }
            // halves combined: one swap per row pair (l, l + NLO/2) leaves row
            // l's total in the lower half and row l + NLO/2's in the upper
            // half, each the row that half writes
#pragma unroll
            for (int l = 0; l < NLO / 2; ++l)
                yb[(l + g * (NLO / 2)) * LS + jh * kE + le] = pair_sum(acc[l], acc[l + NLO / 2]);
        }
        __syncthreads();
        // extinction on the hi patches: thread (lo, e) holds the 2^NH states
        {
            const uint32_t lo = tid / kE;
            if (lo < (uint32_t)NLO) {
                double hv[NHI];
#pragma unroll
                for (int h = 0; h < NHI; ++h) hv[h] = yb[lo * LS + h * kE + le];
#pragma unroll
                for (int k = 0; k < NH; ++k) {
                    const int m = 1 << (NH - 1 - k);
#pragma unroll
                    for (int h = 0; h < NHI; ++h)
                        if (h & m) hv[h] = E * hv[h ^ m] + E1 * hv[h];
                }
#pragma unroll
                for (int h = 0; h < NHI; ++h) y[lo * LS + h * kE + le] = hv[h];
            }
        }
        __syncthreads();
    }
    if (!a.mode) {  // v = P^tdis w, [c][state][e]
        for (uint32_t i = tid; i < (uint32_t)(NS * kE); i += kScnBlock) {
            const uint32_t x = i / kE, l = i % kE, st = ((x % NHI) << NL) | (x / NHI);
            if (e0 + l < a.ne) out[((size_t)ic * NS + st) * a.ne + e0 + l] = y[(x / NHI) * LS + (x % NHI) * kE + l];
        }
        return;
    }
    // L = sum over states: per (lo, e) over hi ascending, then over lo
    {
        const uint32_t lo = tid / kE;
        if (lo < (uint32_t)NLO) {
            double sacc = 0.0;
#pragma unroll
            for (int h = 0; h < NHI; ++h) sacc += y[lo * LS + h * kE + le];
            yb[lo * kE + le] = sacc;
        }
    }
    __syncthreads();
    if (tid < (uint32_t)kE) {
        double L = 0.0;
#pragma unroll
        for (int l = 0; l < NLO; ++l) L += yb[l * kE + tid];
        const uint32_t ie = e0 + tid;
        if (ie < a.ne) out[(((size_t)ie * a.nc + ic) * a.nK + iK) * a.nd + id] = L;
    }
}

// Any n (the reference builds 2^n states for whatever the first row holds,
// dieoff.c:238, loss.c:222): one lane per grid point, its two state vectors
// in an HBM scratch laid out [state][lane] (coalesced).  Per year, for every
// row j (wave-uniform loop, so S[j][k] are scalar loads), the colonisation
// sum over the supersets b of j,
//     (Pc y)[j] = sum_{s <= F} prod_{k in F} (s_k ? pC_jk : 1 - pC_jk) y[j | s],
// F = the patches not in j, is contracted as a binary tree over the free
// patches (lowest state bit innermost) while the supersets stream past in
// ascending order: leaf i completes its trailing-one levels, then parks its
// node as the left child of the next level -- 2^(f+1) flops and 2^f loads
// for a row with f free patches, 2 3^n per year in all.  Then extinction, the
// tensor product over patches, as n in-place pair passes.  Same operator
// order as k_scn (colonisation, then extinction); sums reordered.
__global__ __launch_bounds__(kBigBlock) void k_scn_big(ScnArgs a, const double *__restrict__ S,
                                                       const double *__restrict__ y0src,
                                                       const double *__restrict__ ev, const double *__restrict__ cv,
                                                       const double *__restrict__ Kv, const double *__restrict__ srcv,
                                                       size_t p0, uint32_t npl, double *__restrict__ Y,
                                                       double *__restrict__ out)
{
    typedef const __attribute__((address_space(4))) double cdouble;
    // the contraction's parked left children, per lane: a level index is
    // wave-uniform but dynamic, so LDS rather than (scratch-spilled) registers
    __shared__ double accs[kBigMaxN][kBigBlock];
    double *acc = &accs[0][threadIdx.x];
    const uint32_t q = blockIdx.x * kBigBlock + threadIdx.x;
    const bool live = q < npl;
    const size_t pt = p0 + (live ? q : 0u);
    const uint32_t n = a.n, NS = 1u << n;
    // mode 0: pt = ic ne + ie (v per (c, e)); mode 1: the output order
    uint32_t ie, ic, iK = 0, id = 0;
    if (a.mode) {
        id = (uint32_t)(pt % a.nd);
        iK = (uint32_t)((pt / a.nd) % a.nK);
        ic = (uint32_t)((pt / ((size_t)a.nd * a.nK)) % a.nc);
        ie = (uint32_t)(pt / ((size_t)a.nd * a.nK * a.nc));
    } else {
        ic = (uint32_t)(pt / a.ne);
        ie = (uint32_t)(pt % a.ne);
    }
    const double c = cv[ic], K = a.mode ? Kv[iK] : 1.0;
    const double *src = a.mode && a.loss ? srcv + (size_t)id * n : nullptr;
    const double Kpc = a.mode && !a.loss ? K : 1.0;
    double E = a.mode && !a.loss ? ev[ie] / K : ev[ie];  // dieoff.c:56-57 E = e/K; loss.c:57 E = e
    E = E > 1.0 ? 1.0 : E;
    const double E1 = 1.0 - E;
    const size_t st = (size_t)gridDim.x * kBigBlock;
    double *ya = Y + q, *yb = ya + (size_t)NS * st;
    for (uint32_t s = 0; s < NS; ++s)
        ya[s * st] = a.mode ? y0src[((size_t)ic * NS + s) * a.ne + ie] : y0src[s];
    cdouble *Sc = (cdouble *)S;
    for (int t = 0; t < a.years; ++t) {
        for (uint32_t j = 0; j < NS; ++j) {
            const uint32_t F = ~j & (NS - 1), f = __popc(F);
            // level L = the L-th lowest free state bit, patch n - 1 - bit
            double w0[kBigMaxN], w1[kBigMaxN];
            {
                uint32_t fb = F;
#pragma unroll
                for (uint32_t L = 0; L < kBigMaxN; ++L) {
                    if (!fb) continue;
                    const uint32_t k = n - 1 - (uint32_t)__builtin_ctz(fb);
                    fb &= fb - 1;
                    const double sv = Sc[(size_t)j * n + k];
                    double p = src ? c * (sv + src[k] * K) : c * sv * Kpc;  // dieoff.c:78, loss.c:98
                    p = p > 1.0 ? 1.0 : p;
                    w1[L] = p;
                    w0[L] = 1.0 - p;
                }
            }
            double res = 0.0;
            uint32_t sub = 0;
            for (uint32_t i = 0;; ++i) {
                double cur = ya[(size_t)(j | sub) * st];
                uint32_t L = 0;
                for (; (i >> L) & 1u; ++L) cur = fma(w1[L], cur, acc[L * kBigBlock]);
                if (L == f) {
                    res = cur;
                    break;
                }
                acc[L * kBigBlock] = w0[L] * cur;
                sub = (sub - F) & F;
            }
            yb[(size_t)j * st] = res;
        }
        // extinction, ascending patch: y[s | m] = E y[s] + (1 - E) y[s | m]
        for (uint32_t k = 0; k < n; ++k) {
            const uint32_t m = 1u << (n - 1 - k);
            for (uint32_t s = 0; s < NS; ++s)
                if (s & m) yb[(size_t)s * st] = E * yb[(size_t)(s ^ m) * st] + E1 * yb[(size_t)s * st];
        }
        double *tmp = ya;
        ya = yb;
        yb = tmp;
    }
    if (!live) return;
    if (!a.mode) {
        for (uint32_t s = 0; s < NS; ++s) out[((size_t)ic * NS + s) * a.ne + ie] = ya[(size_t)s * st];
        return;
    }
    double L = 0.0;
    for (uint32_t s = 0; s < NS; ++s) L += ya[(size_t)s * st];
    out[pt] = L;
}

// 8 < n <= 12 (the reference's dieoff / loss on larger first rows,
// dieoff.c:238, loss.c:222, typically one (e, c) and a K grid): one workgroup
// per grid point, its two state vectors in LDS, the 256 threads over the rows
// j.  A row is k_scn_big's contraction -- the supersets of j stream past in
// ascending order and are reduced as a binary tree over the free patches,
// lowest state bit innermost -- with the level factors and parked left
// children in per-thread LDS columns (the level index differs between lanes).
// Rows are dealt round-robin in order of decreasing free-patch count (jord),
// so every thread starts with one of the heavy rows.  Extinction: n in-place
// pair passes, threads over the pairs, a barrier per pass.  Same operator
// order and sums as k_scn_big.
__global__ __launch_bounds__(kRowBlock) void k_scn_row(ScnArgs a, const double *__restrict__ S,
                                                       const double *__restrict__ y0src,
                                                       const double *__restrict__ ev, const double *__restrict__ cv,
                                                       const double *__restrict__ Kv, const double *__restrict__ srcv,
                                                       const uint32_t *__restrict__ jord, size_t p0,
                                                       double *__restrict__ out)
{
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const uint32_t n = a.n, NS = 1u << n, tid = threadIdx.x;
    double *ya = lds, *yb = lds + NS;
    double *accs = lds + 2 * NS;                 // [n][kRowBlock] parked left children
    double *w0s = accs + (size_t)n * kRowBlock;  // [n][kRowBlock] 1 - pC per level
    double *w1s = w0s + (size_t)n * kRowBlock;   // [n][kRowBlock] pC per level
    const size_t pt = p0 + blockIdx.x;
    // mode 0: pt = ic ne + ie (v per (c, e)); mode 1: the output order
    uint32_t ie, ic, iK = 0, id = 0;
    if (a.mode) {
        id = (uint32_t)(pt % a.nd);
        iK = (uint32_t)((pt / a.nd) % a.nK);
        ic = (uint32_t)((pt / ((size_t)a.nd * a.nK)) % a.nc);
        ie = (uint32_t)(pt / ((size_t)a.nd * a.nK * a.nc));
    } else {
        ic = (uint32_t)(pt / a.ne);
        ie = (uint32_t)(pt % a.ne);
    }
    const double c = cv[ic], K = a.mode ? Kv[iK] : 1.0;
    const double *src = a.mode && a.loss ? srcv + (size_t)id * n : nullptr;
    const double Kpc = a.mode && !a.loss ? K : 1.0;
    double E = a.mode && !a.loss ? ev[ie] / K : ev[ie];  // dieoff.c:56-57 E = e/K; loss.c:57 E = e
    E = E > 1.0 ? 1.0 : E;
    const double E1 = 1.0 - E;
    for (uint32_t st = tid; st < NS; st += kRowBlock)
        ya[st] = a.mode ? y0src[((size_t)ic * NS + st) * a.ne + ie] : y0src[st];
    __syncthreads();
    double *acc = accs + tid, *w0 = w0s + tid, *w1 = w1s + tid;
    for (int t = 0; t < a.years; ++t) {
        for (uint32_t r = tid; r < NS; r += kRowBlock) {
            const uint32_t j = jord[r];
            const uint32_t F = ~j & (NS - 1), f = __popc(F);
            {   // level L = the L-th lowest free state bit, patch n - 1 - bit
                uint32_t fb = F;
                for (uint32_t L = 0; L < f; ++L) {
                    const uint32_t k = n - 1 - (uint32_t)__builtin_ctz(fb);
                    fb &= fb - 1;
                    const double sv = S[(size_t)j * n + k];
                    double p = src ? c * (sv + src[k] * K) : c * sv * Kpc;  // dieoff.c:78, loss.c:98
                    p = p > 1.0 ? 1.0 : p;
                    w1[L * kRowBlock] = p;
                    w0[L * kRowBlock] = 1.0 - p;
                }
            }
            double res = 0.0;
            uint32_t sub = 0;
            for (uint32_t i = 0;; ++i) {
                double cur = ya[j | sub];
                uint32_t L = 0;
                for (; (i >> L) & 1u; ++L) cur = fma(w1[L * kRowBlock], cur, acc[L * kRowBlock]);
                if (L == f) {
                    res = cur;
                    break;
                }
                acc[L * kRowBlock] = w0[L * kRowBlock] * cur;
                sub = (sub - F) & F;
            }
            yb[j] = res;
        }
        __syncthreads();
        // extinction, ascending patch: y[s | m] = E y[s] + (1 - E) y[s | m]
        for (uint32_t k = 0; k < n; ++k) {
            const uint32_t m = 1u << (n - 1 - k);
            for (uint32_t q = tid; q < NS / 2; q += kRowBlock) {
                const uint32_t s1 = ((q & ~(m - 1)) << 1) | m | (q & (m - 1));  // q-th state with bit m set
                yb[s1] = E * yb[s1 ^ m] + E1 * yb[s1];
            }
            __syncthreads();
        }
        double *tmp = ya;
        ya = yb;
        yb = tmp;
    }
    if (!a.mode) {
        for (uint32_t st = tid; st < NS; st += kRowBlock) out[((size_t)ic * NS + st) * a.ne + ie] = ya[st];
        return;
    }
    // L = sum over the states: per thread a strided partial, then thread 0
    // adds the 256 partials in order
    double part = 0.0;
    for (uint32_t st = tid; st < NS; st += kRowBlock) part += ya[st];
    acc[0] = part;
    __syncthreads();
    if (tid == 0) {
        double L = 0.0;
        for (int i = 0; i < kRowBlock; ++i) L += accs[i];
        out[pt] = L;
    }
}

size_t row_lds(uint32_t n) { return (2 * ((size_t)1 << n) + 3 * (size_t)n * kRowBlock) * sizeof(double); }

// instantiation for n patches: NL = min(3, n) lo patches, NH = n - NL
typedef void (*ScnKernel)(ScnArgs, const double *, const double *, const double *, const double *, const double *,
                          const double *, const uint32_t *, const uint32_t *, double *);
ScnKernel scn_kernel(uint32_t n)
{
    switch (n) {
    case 1: return k_scn<1, 0>;
    case 2: return k_scn<2, 0>;
    case 3: return k_scn<3, 0>;
    case 4: return k_scn<3, 1>;
    case 5: return k_scn<3, 2>;
    case 6: return k_scn<3, 3>;
    case 7: return k_scn<3, 4>;
    case 8: return k_scn<3, 5>;
    default: return nullptr;
    }
}
uint32_t scn_nl(uint32_t n) { return n < 3 ? n : 3u; }

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
    uint32_t n = 0, ns = 0;
    int kind = 0;  // 0 die-off, 1 habitat loss
    double m = 400.0, d = 200.0;
    int device = 0;
    std::vector<double> S, w;
    std::vector<uint32_t> boff, jsched;  // hi factor table offsets; per-wave hi-row schedule
    uint32_t nsched = 0, btot = 0;
    double *dS = nullptr, *dw = nullptr;
    uint32_t *dboff = nullptr, *djsched = nullptr;
    hipStream_t stream = nullptr;
    // grid set by mdp_scenario_set_grid (device resident)
    int ts = 0, tdis = 0;
    uint32_t ne = 0, nc = 0, nK = 0, nd = 0;
    double *de = nullptr, *dc = nullptr, *dK = nullptr, *dsr = nullptr, *dV = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // k_scn_big (n > 8, or MDP_SCN_BIG=1): state-vector scratch, points per launch
    bool big = false;
    double *dY = nullptr;
    uint32_t big_pts = 0;
    // k_scn_row (8 < n <= 12, or MDP_SCN_ROW=1): rows by decreasing free-patch count
    bool row = false;
    uint32_t *djord = nullptr;
};

namespace {

void scn_free_grid(mdp_scenario *sc)
{
    for (double **p : {&sc->de, &sc->dc, &sc->dK, &sc->dsr, &sc->dV, &sc->dY}) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
    sc->ne = sc->nc = sc->nK = sc->nd = 0;
}

size_t scn_lds(const mdp_scenario *sc)
{
    const uint32_t nl = scn_nl(sc->n), nh = sc->n - nl;
    const size_t na = (size_t)((pow3((int)nl) + 1) & ~1) << nh;
    return (2 * ((size_t)sc->ns * kE + (2u << nl)) + na + sc->btot + (1u << nl)) * sizeof(double);
}

// v = P^tdis w (which = 1), L = 1^T PK^ts v (which = 2) or both (3) on stream st
int scn_launch(mdp_scenario *sc, double *dout, hipStream_t st, int which)
{
    if (sc->row) {
        for (int mode = 0; mode < 2; ++mode) {
            if (!(which & (1 << mode))) continue;
            ScnArgs a{sc->n, sc->ns, sc->ne, sc->nc, sc->nK, sc->nd, mode ? sc->ts : sc->tdis, sc->kind, mode, 0, 0};
            const double *y0 = mode ? sc->dV : sc->dw;
            double *o = mode ? dout : sc->dV;
            const size_t tot = mode ? (size_t)sc->ne * sc->nc * sc->nK * sc->nd : (size_t)sc->nc * sc->ne;
            constexpr size_t kPer = (size_t)1 << 22;  // points per launch (grid of < 2^32 threads)
            for (size_t p0 = 0; p0 < tot; p0 += kPer) {  // one workgroup per point
                const uint32_t nb = (uint32_t)std::min(kPer, tot - p0);
                hipLaunchKernelGGL(k_scn_row, dim3(nb), dim3(kRowBlock), row_lds(sc->n), st, a, sc->dS, y0, sc->de,
                                   sc->dc, sc->dK, sc->dsr, sc->djord, p0, o);
            }
            SCN_TRY(hipGetLastError());
        }
        return MDP_OK;
    }
    if (sc->big) {
        for (int mode = 0; mode < 2; ++mode) {
            if (!(which & (1 << mode))) continue;
            ScnArgs a{sc->n, sc->ns, sc->ne, sc->nc, sc->nK, sc->nd, mode ? sc->ts : sc->tdis, sc->kind, mode, 0, 0};
            const double *y0 = mode ? sc->dV : sc->dw;
            double *o = mode ? dout : sc->dV;
            const size_t tot = mode ? (size_t)sc->ne * sc->nc * sc->nK * sc->nd : (size_t)sc->nc * sc->ne;
            for (size_t p0 = 0; p0 < tot; p0 += sc->big_pts) {
                const uint32_t npl = (uint32_t)std::min<size_t>(sc->big_pts, tot - p0);
                hipLaunchKernelGGL(k_scn_big, dim3(sc->big_pts / kBigBlock), dim3(kBigBlock), 0, st, a, sc->dS, y0,
                                   sc->de, sc->dc, sc->dK, sc->dsr, p0, npl, sc->dY, o);
            }
            SCN_TRY(hipGetLastError());
        }
        return MDP_OK;
    }
    const uint32_t nchunk = (sc->ne + kE - 1) / kE;
    ScnKernel fn = scn_kernel(sc->n);
    const size_t lds = scn_lds(sc);
    const size_t npt = (size_t)sc->nc * sc->nK * sc->nd;
    for (int mode = 0; mode < 2; ++mode) {
        if (!(which & (1 << mode))) continue;
        ScnArgs a{sc->n, sc->ns, sc->ne, sc->nc, sc->nK, sc->nd, mode ? sc->ts : sc->tdis, sc->kind, mode,
                  sc->nsched, sc->btot};
        const double *y0 = mode ? sc->dV : sc->dw;
        double *o = mode ? dout : sc->dV;
        void *args[] = {&a, &sc->dS, &y0, &sc->de, &sc->dc, &sc->dK, &sc->dsr, &sc->dboff, &sc->djsched, &o};
        const uint32_t nb = (uint32_t)(nchunk * (mode ? npt : sc->nc));
        SCN_TRY(hipLaunchKernel((const void *)fn, dim3(nb), dim3(kScnBlock), args, lds, st));
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

int mdp_device_count(void)
{
    int ndev = 0;
    return hipGetDeviceCount(&ndev) == hipSuccess ? ndev : 0;
}

int mdp_scenario_create(const int32_t *row, uint32_t n, double m, float p, double d, int kind, int device,
                        mdp_scenario **out)
{
    return mdp_scenario_create_opts(row, n, m, p, d, kind, device, nullptr, out);
}

// options (ABI 7): "MDP_SCN_BIG=1" / "MDP_SCN_ROW=1" force the HBM-state or
// the row-parallel kernel (tests pin the kernels against each other); the
// library reads no environment
int mdp_scenario_create_opts(const int32_t *row, uint32_t n, double m, float p, double d, int kind, int device,
                             const char *options, mdp_scenario **out)
{
    if (!row || !out || n == 0) return mdp_set_error(MDP_EINVAL, "null argument");
    *out = nullptr;
    bool force_big = false, force_row = false;
    if (options) {
        std::string cur;
        for (const char *c = options;; ++c) {
            if (*c == 0 || *c == ';' || *c == ',' || *c == ' ' || *c == '\t' || *c == '\n') {
                if (!cur.empty()) {
                    const size_t eq = cur.find('=');
                    const std::string k = cur.substr(0, eq);
                    const bool on = eq == std::string::npos || atoi(cur.c_str() + eq + 1) != 0;
                    if (k == "MDP_SCN_BIG") force_big = on;
                    else if (k == "MDP_SCN_ROW") force_row = on;
                    else return mdp_set_error(MDP_EINVAL, "unknown scenario option '%s'", k.c_str());
                    cur.clear();
                }
                if (*c == 0) break;
            } else {
                cur += *c;
            }
        }
    }
    if (n > kBigMaxN)
        return mdp_set_error(MDP_EUNSUPPORTED, "%u patches: the scenario engine takes n <= %u (2^n states)", n,
                             kBigMaxN);
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
    // n > 8: the LDS-resident k_scn does not fit; 8 < n <= 12: k_scn_row
    // (option MDP_SCN_ROW=1 forces it for any n <= 12); n > 12: k_scn_big
    // (MDP_SCN_BIG=1 forces it for any n)
    sc->row = !force_big && n <= kRowMaxN && (n > kMaxN || force_row);
    sc->big = !sc->row && (n > kMaxN || force_big);
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
    // hi factor table offsets (rows jh ascending, 2^(NH-|jh|) supersets x
    // 2^NL lo rows each) and the hi-row schedule: rows dealt to the waves by
    // longest-processing-time-first (row jh costs its 2^(f-1) superset
    // pairs, f = NH - |jh|, plus one for its loads and epilogue)
    std::vector<uint32_t> jord;
    if (sc->row) {  // rows by decreasing free-patch count (stable: ascending j within a count)
        jord.resize(ns);
        for (uint32_t j = 0; j < ns; ++j) jord[j] = j;
        std::stable_sort(jord.begin(), jord.end(),
                         [](uint32_t x, uint32_t y) { return __builtin_popcount(x) < __builtin_popcount(y); });
    }
    if (!sc->big && !sc->row) {
        const uint32_t nl = scn_nl(n), nh = n - nl, nhi = 1u << nh;
        sc->boff.assign(nhi, 0);
        uint32_t off = 0;
        for (uint32_t jh = 0; jh < nhi; ++jh) {
            sc->boff[jh] = off;
            off += (1u << (nh - __builtin_popcount(jh))) << nl;
        }
        sc->btot = off;
        std::vector<uint32_t> rows(nhi);
        for (uint32_t jh = 0; jh < nhi; ++jh) rows[jh] = jh;
        auto cost = [&](uint32_t jh) {
            const uint32_t f = nh - __builtin_popcount(jh);
            return (f ? 1u << (f - 1) : 1u) + 1u;
        };
        std::stable_sort(rows.begin(), rows.end(), [&](uint32_t x, uint32_t y) { return cost(x) > cost(y); });
        std::vector<std::vector<uint32_t>> grp(kWaves);
        std::vector<uint64_t> load(kWaves, 0);
        for (uint32_t jh : rows) {
            const size_t g = (size_t)(std::min_element(load.begin(), load.end()) - load.begin());
            grp[g].push_back(jh);
            load[g] += cost(jh);
        }
        size_t mx = 0;
        for (auto &v : grp) mx = std::max(mx, v.size());
        sc->nsched = (uint32_t)mx;
        sc->jsched.assign(mx * kWaves, 0xffffffffu);
        for (uint32_t g = 0; g < (uint32_t)kWaves; ++g)
            for (size_t i = 0; i < grp[g].size(); ++i) sc->jsched[g * mx + i] = grp[g][i];
    }
    int rc;
    if (hipSetDevice(device) != hipSuccess) {
        delete sc;
        return mdp_set_error(MDP_EHIP, "hipSetDevice(%d) failed", device);
    }
    if ((rc = dev_up(&sc->dS, sc->S)) || (rc = dev_up(&sc->dw, sc->w)) || (rc = dev_up(&sc->dboff, sc->boff)) ||
        (rc = dev_up(&sc->djsched, sc->jsched)) || (rc = dev_up(&sc->djord, jord)) ||
        hipStreamCreateWithFlags(&sc->stream, hipStreamNonBlocking) != hipSuccess) {
        mdp_scenario_destroy(sc);
        return rc ? rc : mdp_set_error(MDP_EHIP, "stream creation failed");
    }
    if (sc->row) {
        if (row_lds(n) > 64 * 1024)
            (void)hipFuncSetAttribute((const void *)k_scn_row, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)row_lds(n));
    } else if (!sc->big) {
        const size_t lds = scn_lds(sc);
        if (lds > 64 * 1024)
            (void)hipFuncSetAttribute((const void *)scn_kernel(n), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
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
    for (void *p : {(void *)sc->dS, (void *)sc->dw, (void *)sc->dboff, (void *)sc->djsched, (void *)sc->djord})
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
        hipMalloc((void **)&sc->dV, (size_t)nc * ns * ne * sizeof(double)) != hipSuccess) {
        scn_free_grid(sc);
        return mdp_set_error(MDP_ENOMEM, "device allocation failed");
    }
    if (sc->big) {  // points per k_scn_big launch: two state vectors each within kBigScratch
        const size_t tot = std::max((size_t)ne * nc * nK * nd, (size_t)nc * ne);
        size_t pts = kBigScratch / (2 * (size_t)ns * sizeof(double));
        pts = std::max<size_t>(kBigBlock, std::min(pts, tot + kBigBlock - 1) / kBigBlock * kBigBlock);
        sc->big_pts = (uint32_t)std::min<size_t>(pts, (size_t)65535 * kBigBlock);
        if (hipMalloc((void **)&sc->dY, 2 * (size_t)ns * sc->big_pts * sizeof(double)) != hipSuccess) {
            scn_free_grid(sc);
            return mdp_set_error(MDP_ENOMEM, "device allocation failed (state scratch)");
        }
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
    return scn_launch(sc, d_out, (hipStream_t)stream, 3);
}

int mdp_scenario_time_kernels(mdp_scenario *sc, double *d_out, void *stream, int reps, double *ms)
{
    if (!sc || !ms || reps <= 0) return mdp_set_error(MDP_EINVAL, "bad timing request");
    if (!sc->ne) return mdp_set_error(MDP_EINVAL, "no grid set");
    SCN_TRY(hipSetDevice(sc->device));
    hipStream_t st = (hipStream_t)stream;
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
