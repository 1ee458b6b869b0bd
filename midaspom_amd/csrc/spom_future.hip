// midaspom_amd/csrc/spom_future.hip -- MI355X engine for the reference's
// forward-simulation program MIDASPOM_future:
//   /root/reference/sources/main_MIDASPOM_future.c:343-386  (replicate loop)
//   /root/reference/sources/main_MIDASPOM_future.c:64-110   (simpij: one year)
//
// Every replicate
//   1. samples (e, c) from the trapezoid-weighted posterior by inverse CDF on
//      the (necstep-1)^2 scale with the hard-coded e = ie*0.01, c = ic*0.01
//      (:361-375); a draw above the last cumulative value keeps the previous
//      replicate's (e, c) (the goto is skipped), (0, 0) before the first;
//   2. picks the initial state uniformly among the missing-data completions
//      of the last survey row (:378-379);
//   3. simulates tfut years of extinction (E = e/K_D) then colonisation
//      (pC = min(1, c*(sum_{l occupied, l != k} M[l][k]*K_D + M[n][k]*K_S)))
//      and counts, per year, the replicates with every patch empty (:381-385).
//
// GPU design: one lane per replicate (grid-stride over replicates, >= 8
// waves per CU), the occupancy of all patches as one 64-bit mask in a VGPR,
// the colonisation sums in registers (a template over the padded patch
// count), the M*K_D table read with uniform addresses (scalar loads), and
// the per-year all-extinct counts aggregated by wave ballots into LDS, then
// per workgroup into a partial table reduced by k_future_sum (integer sums,
// deterministic).
//
// Random numbers: the reference draws rand()/RAND_MAX from one sequential
// stream per process (srand(time(NULL)), :345).  Here every draw is
// addressed -- Philox4x32-10 keyed by the 64-bit seed, counter (replicate,
// year, patch pair) -- so a replicate's trajectory is independent of how
// replicates are split over lanes, workgroups or GPUs.  A draw is the high
// 31 bits of a Philox word r, used exactly as the reference uses rand():
// u = (double)r / (double)RAND_MAX, init = r % npstates.  Word layout of
// philox(key, {rep_lo, rep_hi, t, k >> 1}): [2*(k&1)] extinction draw of
// patch k, [2*(k&1)+1] its colonisation draw; counter {rep_lo, rep_hi,
// 0xffffffff, 0}: word 0 the posterior draw, word 1 the initial state.  The
// CPU restatement (oracle/spom_future_oracle.c) uses the same stream, so the
// counts agree bit for bit; with glibc rand() it reproduces the reference's
// own sequential stream (statistical parity, tests/test_future_oracle.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "mdp_internal.h"

#pragma clang fp contract(off)

namespace {

constexpr int kFutBlock = 256;
constexpr int kFutMaxWG = 4096;         // grid-stride cap (>= 16 workgroups per CU)
constexpr uint32_t kFutMaxT = 12288;    // LDS year counters (48 KB; + 16 KB table for n <= 8)
constexpr uint32_t kLookBack = 1u << 16;
constexpr double kRandMax = 2147483647.0;  // glibc RAND_MAX

#define FUT_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return mdp_set_error(MDP_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                                 __FILE__, __LINE__);                                        \
    } while (0)

// Philox4x32-10 (Salmon et al., SC'11), the Random123 constants.
struct u32x4 {
    uint32_t x, y, z, w;
};

__device__ __forceinline__ u32x4 philox(uint32_t k0, uint32_t k1, u32x4 c)
{
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        // one v_mad_u64_u32 per product (instead of mul_lo + mul_hi)
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

struct FutArgs {
    uint32_t n, nmiss, tfut, lvalid;
    uint64_t occ0;          // bit k = patch k occupied in the last survey (:315-316)
    uint64_t rep0, nrep;    // global index of the first replicate, count
    uint32_t key0, key1;    // seed
    uint32_t necstep, pad;
    double pscale;          // (double)((necstep-1)*(necstep-1)) (:361)
    double K;               // K_D (:67, :93)
};

// The reference compares u = (double)r / (double)RAND_MAX with a threshold
// (u > E, u < pC).  r * fl(1/RAND_MAX) is within 3.4e-16 of fl(r/RAND_MAX)
// (both within ~1.2 ulp of r/RAND_MAX <= 1), so outside a 1e-15 band around
// the threshold the product decides the comparison; inside it the exact
// correctly rounded quotient does.  Bit-identical outcomes, ~never divides.
constexpr double kInvRandMax = 1.0 / 2147483647.0;
constexpr double kBand = 1e-15;

__device__ __forceinline__ bool u_gt(uint32_t r, double x)  // fl(r/R) > x
{
    const double q = (double)r * kInvRandMax;
    if (q > x + kBand) return true;
    if (q < x - kBand) return false;
    return (double)r / kRandMax > x;
}

__device__ __forceinline__ bool u_lt(uint32_t r, double x)  // fl(r/R) < x
{
    const double q = (double)r * kInvRandMax;
    if (q < x - kBand) return true;
    if (q > x + kBand) return false;
    return (double)r / kRandMax < x;
}

// first i < len with x < pcum[i] (pcum non-decreasing), or len
__device__ __forceinline__ uint32_t upper_bound(const double *__restrict__ pcum, uint32_t len, double x)
{
    uint32_t lo = 0, cnt = len;
    while (cnt > 0) {
        const uint32_t half = cnt >> 1, mid = lo + half;
        if (!(x < pcum[mid])) lo = mid + 1, cnt -= half + 1;
        else cnt = half;
    }
    return lo;
}

// colonisation sums of every survivor set of n <= 8 patches:
// T[surv][k] = (sum_{l in surv, l != k, ascending} M[l][k]*K_D) + M[n][k]*K_S,
// the reference's s1 of simpij :89-95 (its added zeros change nothing)
constexpr int kTabN = 8;
__global__ __launch_bounds__(256) void k_future_table(const double *__restrict__ MK, const double *__restrict__ src,
                                                      uint32_t n, double *__restrict__ T)
{
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= (1u << kTabN) * kTabN) return;
    const uint32_t surv = i / kTabN, k = i % kTabN;
    double s1 = 0.0;
    for (uint32_t l = 0; l < n; ++l)
        if (l != k && ((surv >> l) & 1u)) s1 += MK[l * kTabN + k];
    T[i] = s1 + src[k];
}

template <int NM>
__global__ __launch_bounds__(kFutBlock) void k_future(FutArgs a, const double *__restrict__ MK,
                                                      const double *__restrict__ src,
                                                      const double *__restrict__ pcum,
                                                      const uint64_t *__restrict__ missbit,
                                                      const double *__restrict__ T,
                                                      uint32_t *__restrict__ partial, uint32_t *__restrict__ err)
{
    extern __shared__ __attribute__((aligned(16))) double dyn[];
    // NM == 8: the colonisation table (16 KB) first, then the year counters
    double *Ts = dyn;
    uint32_t *cnt = (uint32_t *)(dyn + (NM == kTabN ? (1 << kTabN) * kTabN : 0));
    if constexpr (NM == kTabN) {
        for (uint32_t i = threadIdx.x; i < (1u << kTabN) * kTabN / 2; i += kFutBlock)
            reinterpret_cast<double2 *>(Ts)[i] = reinterpret_cast<const double2 *>(T)[i];
    }
    for (uint32_t t = threadIdx.x; t < a.tfut; t += kFutBlock) cnt[t] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t npairs = (a.n + 1) >> 1;
    for (uint64_t r = (uint64_t)blockIdx.x * kFutBlock + threadIdx.x; r < a.nrep;
         r += (uint64_t)gridDim.x * kFutBlock) {
        const uint64_t rg = a.rep0 + r;
        // ---- (e, c) from the posterior, with the reference's carry-over (:361-377)
        uint32_t idx = a.lvalid, init_w = 0;
        {
            uint64_t q = rg;
            for (uint32_t step = 0;; ++step) {
                const u32x4 w = philox(a.key0, a.key1, u32x4{(uint32_t)q, (uint32_t)(q >> 32), 0xffffffffu, 0u});
                if (step == 0) init_w = w.y >> 1;
                if (a.lvalid == 0) break;  // empty / all-NaN posterior: never found
                const double pec = a.pscale * (double)(w.x >> 1) / kRandMax;
                idx = upper_bound(pcum, a.lvalid, pec);
                if (idx < a.lvalid || q == 0) break;
                if (step + 1 >= kLookBack) {  // posterior mass too small for an exact look-back
                    atomicOr(err, 1u);
                    break;
                }
                --q;
            }
        }
        uint32_t ie = 0, ic = 0;
        if (idx < a.lvalid) ie = idx / a.necstep, ic = idx - ie * a.necstep;
        const double e = (double)ie * 0.01, c = (double)ic * 0.01;
        double E = e / a.K;  // simpij :67, :74
        if (E > 1) E = 1;
        // ---- initial state: missing columns filled from init (first missing = MSB) (:315-321, :378)
        const uint32_t init = init_w & ((1u << a.nmiss) - 1u);
        uint64_t occ = a.occ0;
        for (uint32_t q = 0; q < a.nmiss; ++q)
            if ((init >> (a.nmiss - 1 - q)) & 1u) occ |= missbit[q];
        // ---- tfut years (:381-385)
        for (uint32_t t = 0; t < a.tfut; ++t) {
            uint64_t surv = 0;
            uint32_t colw[NM];
#pragma unroll
            for (int m = 0; m < NM / 2; ++m) {
                if ((uint32_t)m < npairs) {
                    const u32x4 w = philox(a.key0, a.key1, u32x4{(uint32_t)rg, (uint32_t)(rg >> 32), t, (uint32_t)m});
                    const uint32_t k0 = 2 * m, k1 = 2 * m + 1;
                    colw[k0] = w.y >> 1;
                    colw[k1] = w.w >> 1;
                    // extinction: an occupied patch survives if u > E (:75-82)
                    if (((occ >> k0) & 1u) && u_gt(w.x >> 1, E)) surv |= 1ull << k0;
                    if (((occ >> k1) & 1u) && u_gt(w.z >> 1, E)) surv |= 1ull << k1;
                } else {
                    colw[2 * m] = colw[2 * m + 1] = 0;
                }
            }
            // colonisation sums, ascending l for every k (:89-95)
            double s1[NM];
            if constexpr (NM == kTabN) {
                const double2 *row = reinterpret_cast<const double2 *>(Ts + (uint32_t)surv * kTabN);
#pragma unroll
                for (int k = 0; k < NM; k += 2) {
                    const double2 v = row[k / 2];
                    s1[k] = v.x, s1[k + 1] = v.y;
                }
            } else {
#pragma unroll
                for (int k = 0; k < NM; ++k) s1[k] = 0.0;
                for (uint32_t l = 0; l < a.n; ++l) {
                    const bool on = (surv >> l) & 1u;
#pragma unroll
                    for (int k = 0; k < NM; ++k) s1[k] += on ? MK[l * NM + k] : 0.0;
                }
#pragma unroll
                for (int k = 0; k < NM; ++k) s1[k] += src[k];
            }
            uint64_t nw = surv;
#pragma unroll
            for (int k = 0; k < NM; ++k) {
                if ((uint32_t)k < a.n && !((surv >> k) & 1u)) {
                    double pc = c * s1[k];  // :95-97
                    if (pc > 1) pc = 1;
                    if (u_lt(colw[k], pc)) nw |= 1ull << k;  // :98-101
                }
            }
            occ = nw;
            const uint64_t ext = __ballot(occ == 0);
            if (ext && lane == (uint32_t)(__ffsll((unsigned long long)__ballot(1)) - 1))
                atomicAdd(&cnt[t], (uint32_t)__popcll(ext));
        }
    }
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < a.tfut; t += kFutBlock) partial[(size_t)blockIdx.x * a.tfut + t] = cnt[t];
}

// counts[t] = sum over workgroups of partial[wg][t]  (one workgroup per year)
__global__ __launch_bounds__(256) void k_future_sum(const uint32_t *__restrict__ partial, uint32_t nwg, uint32_t tfut,
                                                    unsigned long long *__restrict__ counts)
{
    __shared__ unsigned long long red[256];
    const uint32_t t = blockIdx.x;
    unsigned long long s = 0;
    for (uint32_t b = threadIdx.x; b < nwg; b += 256) s += partial[(size_t)b * tfut + t];
    red[threadIdx.x] = s;
    __syncthreads();
    for (uint32_t w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) counts[t] = red[0];
}

template <typename T>
int dev_up(T **p, const std::vector<T> &h)
{
    FUT_TRY(hipMalloc((void **)p, std::max<size_t>(1, h.size()) * sizeof(T)));
    if (!h.empty()) FUT_TRY(hipMemcpy(*p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return MDP_OK;
}

}  // namespace

struct mdp_future {
    int device = 0;
    uint32_t n = 0, nm = 0, nmiss = 0, necstep = 0, lvalid = 0;
    uint64_t occ0 = 0;
    double K = 1.0, pscale = 0.0;
    double *dMK = nullptr, *dsrc = nullptr, *dpcum = nullptr, *dT = nullptr;
    uint64_t *dmiss = nullptr;
    uint32_t *dpartial = nullptr, *derr = nullptr;
    size_t partial_cap = 0;
    unsigned long long *dcounts = nullptr;
    size_t counts_cap = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
};

namespace {

int fut_grid(uint64_t nrep)
{
    const uint64_t wg = (nrep + kFutBlock - 1) / kFutBlock;
    return (int)std::max<uint64_t>(1, std::min<uint64_t>(wg, kFutMaxWG));
}

int fut_reserve(mdp_future *f, int nwg, uint32_t tfut)
{
    const size_t need = (size_t)nwg * tfut;
    if (need > f->partial_cap) {
        if (f->dpartial) (void)hipFree(f->dpartial);
        f->dpartial = nullptr;
        f->partial_cap = 0;
        FUT_TRY(hipMalloc((void **)&f->dpartial, need * sizeof(uint32_t)));
        f->partial_cap = need;
    }
    if (tfut > f->counts_cap) {
        if (f->dcounts) (void)hipFree(f->dcounts);
        f->dcounts = nullptr;
        f->counts_cap = 0;
        FUT_TRY(hipMalloc((void **)&f->dcounts, tfut * sizeof(unsigned long long)));
        f->counts_cap = tfut;
    }
    return MDP_OK;
}

// one simulation (k_future + k_future_sum) into d_counts on stream st
int fut_launch(mdp_future *f, uint64_t seed, uint64_t rep0, uint64_t nrep, uint32_t tfut,
               unsigned long long *d_counts, hipStream_t st, bool sum, uint32_t *derr)
{
    FutArgs a{};
    a.n = f->n;
    a.nmiss = f->nmiss;
    a.tfut = tfut;
    a.lvalid = f->lvalid;
    a.occ0 = f->occ0;
    a.rep0 = rep0;
    a.nrep = nrep;
    a.key0 = (uint32_t)seed;
    a.key1 = (uint32_t)(seed >> 32);
    a.necstep = f->necstep;
    a.pscale = f->pscale;
    a.K = f->K;
    const int nwg = fut_grid(nrep);
    const size_t lds = (size_t)tfut * sizeof(uint32_t) + (f->nm == kTabN ? sizeof(double) * (kTabN << kTabN) : 0);
    switch (f->nm) {
#define FUT_CASE(NMV)                                                                                   \
    case NMV:                                                                                            \
        hipLaunchKernelGGL(k_future<NMV>, dim3(nwg), dim3(kFutBlock), lds, st, a, f->dMK, f->dsrc,    \
                           f->dpcum, f->dmiss, f->dT, f->dpartial, derr);                               \
        break;
        FUT_CASE(8)
        FUT_CASE(16)
        FUT_CASE(32)
        FUT_CASE(64)
#undef FUT_CASE
    default:
        return mdp_set_error(MDP_EINVAL, "internal: padded patch count %u", f->nm);
    }
    FUT_TRY(hipGetLastError());
    if (sum) {
        hipLaunchKernelGGL(k_future_sum, dim3(tfut), dim3(256), 0, st, f->dpartial, (uint32_t)nwg, tfut, d_counts);
        FUT_TRY(hipGetLastError());
    }
    return MDP_OK;
}

int fut_check_args(mdp_future *f, uint64_t nrep, uint32_t tfut)
{
    if (!f) return mdp_set_error(MDP_EINVAL, "null future engine");
    if (tfut == 0 || tfut > kFutMaxT)
        return mdp_set_error(MDP_EUNSUPPORTED, "duration %u outside 1..%u years", tfut, kFutMaxT);
    if (nrep > (1ull << 62)) return mdp_set_error(MDP_EINVAL, "replicate count too large");
    return MDP_OK;
}

}  // namespace

extern "C" {

int mdp_future_create(const int32_t *last_row, uint32_t n, const double *post, uint32_t necstep, double m,
                      double d, double KD, double KS, double dS, int device, mdp_future **out)
{
    if (!last_row || !out || n == 0) return mdp_set_error(MDP_EINVAL, "empty survey row");
    if (n > 64) return mdp_set_error(MDP_EUNSUPPORTED, "%u patches: the future engine holds <= 64", n);
    if (necstep > 0 && !post) return mdp_set_error(MDP_EINVAL, "null posterior");
    if (!(KD >= 0) || !std::isfinite(KD) || !(KS >= 0) || !std::isfinite(KS))
        return mdp_set_error(MDP_EINVAL, "-D and -S must be finite and >= 0");
    if (!(m > 0) && !(m < 0)) return mdp_set_error(MDP_EINVAL, "mean dispersal -m must be non-zero");
    mdp_future *f = new (std::nothrow) mdp_future();
    if (!f) return mdp_set_error(MDP_ENOMEM, "out of host memory");
    f->device = device;
    f->n = n;
    f->nm = n <= 8 ? 8 : n <= 16 ? 16 : n <= 32 ? 32 : 64;
    f->K = KD;
    f->necstep = necstep;
    // last survey row -> occupied bits and missing columns (:292-323)
    std::vector<uint64_t> miss;
    for (uint32_t j = 0; j < n; ++j) {
        if (last_row[j] == 1) f->occ0 |= 1ull << j;
        else if (last_row[j] == -1) miss.push_back(1ull << j);
        else if (last_row[j] != 0) {
            delete f;
            return mdp_set_error(MDP_EINVAL, "survey value %d in column %u (expected -1, 0 or 1)", last_row[j], j);
        }
    }
    if (miss.size() > 30) {
        delete f;
        return mdp_set_error(MDP_EUNSUPPORTED, "%zu missing patches (npstates = 2^%zu overflows int)", miss.size(),
                             miss.size());
    }
    f->nmiss = (uint32_t)miss.size();
    // dispersal (:266-277), a = 1/m; M*K_D and the source term M[n][k]*K_S
    const double a = 1.0 / m;
    std::vector<double> MK((size_t)f->nm * f->nm, 0.0), src(f->nm, 0.0);
    for (uint32_t i = 0; i < n; ++i)
        for (uint32_t j = i + 1; j < n; ++j) {
            const double v = exp(-a * (j - i) * d);
            MK[(size_t)i * f->nm + j] = v * KD;
            MK[(size_t)j * f->nm + i] = v * KD;
        }
    for (uint32_t j = 0; j < n; ++j) src[j] = exp(-a * (j + 1) * dS) * KS;
    // trapezoid-weighted cumulative posterior in the reference's scan order
    // (:362-369); the scan stops matching at the first NaN
    std::vector<double> pcum((size_t)necstep * necstep);
    double acc = 0;
    size_t lv = pcum.size();
    for (uint32_t ie = 0; ie < necstep; ++ie)
        for (uint32_t ic = 0; ic < necstep; ++ic) {
            double w = 1.0;
            if (ie == 0 || ie == necstep - 1) w *= 0.5;
            if (ic == 0 || ic == necstep - 1) w *= 0.5;
            acc += w * post[(size_t)ie * necstep + ic];
            const size_t i = (size_t)ie * necstep + ic;
            pcum[i] = acc;
            if (std::isnan(acc) && lv == pcum.size()) lv = i;
        }
    for (size_t i = 1; i < lv; ++i)
        if (pcum[i] < pcum[i - 1]) {
            delete f;
            return mdp_set_error(MDP_EUNSUPPORTED, "posterior with negative entries (cell %zu): the sampler "
                                 "needs a non-decreasing cumulative sum", i);
        }
    if (lv > 0 && !(pcum[lv - 1] > 0)) lv = 0;  // no draw is ever below the mass: (0, 0) for all
    f->lvalid = (uint32_t)lv;
    f->pscale = (double)((int)(necstep - 1) * (int)(necstep - 1));
    int rc;
    if (hipSetDevice(device) != hipSuccess) {
        delete f;
        return mdp_set_error(MDP_EHIP, "hipSetDevice(%d) failed", device);
    }
    if ((rc = dev_up(&f->dMK, MK)) || (rc = dev_up(&f->dsrc, src)) || (rc = dev_up(&f->dpcum, pcum)) ||
        (rc = dev_up(&f->dmiss, miss))) {
        mdp_future_destroy(f);
        return rc;
    }
    if (f->nm == kTabN) {
        if (hipMalloc((void **)&f->dT, sizeof(double) * (kTabN << kTabN)) != hipSuccess) {
            mdp_future_destroy(f);
            return mdp_set_error(MDP_EHIP, "device allocation failed on device %d", device);
        }
        hipLaunchKernelGGL(k_future_table, dim3((kTabN << kTabN) / 256), dim3(256), 0, nullptr, f->dMK, f->dsrc, n,
                           f->dT);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
            mdp_future_destroy(f);
            return mdp_set_error(MDP_EHIP, "colonisation table kernel failed on device %d", device);
        }
    }
    // look-back overflow flags: [0] the device path (read and cleared by
    // mdp_future_check), [1] the host-returning calls (their own)
    if (hipMalloc((void **)&f->derr, 2 * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(f->derr, 0, 2 * sizeof(uint32_t)) != hipSuccess ||
        hipStreamCreateWithFlags(&f->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&f->ev0) != hipSuccess || hipEventCreate(&f->ev1) != hipSuccess) {
        mdp_future_destroy(f);
        return mdp_set_error(MDP_EHIP, "device setup failed on device %d", device);
    }
    *out = f;
    return MDP_OK;
}

void mdp_future_destroy(mdp_future *f)
{
    if (!f) return;
    (void)hipSetDevice(f->device);
    if (f->stream) (void)hipStreamSynchronize(f->stream);
    (void)hipFree(f->dMK);
    (void)hipFree(f->dsrc);
    (void)hipFree(f->dpcum);
    (void)hipFree(f->dT);
    (void)hipFree(f->dmiss);
    (void)hipFree(f->dpartial);
    (void)hipFree(f->derr);
    (void)hipFree(f->dcounts);
    if (f->ev0) (void)hipEventDestroy(f->ev0);
    if (f->ev1) (void)hipEventDestroy(f->ev1);
    if (f->stream) (void)hipStreamDestroy(f->stream);
    delete f;
}

int mdp_future_simulate_device(mdp_future *f, uint64_t seed, uint64_t rep0, uint64_t nrep, uint32_t tfut,
                               uint64_t *d_counts, void *stream)
{
    int rc = fut_check_args(f, nrep, tfut);
    if (rc) return rc;
    if (!d_counts) return mdp_set_error(MDP_EINVAL, "null device counts");
    FUT_TRY(hipSetDevice(f->device));
    hipStream_t st = (hipStream_t)stream;  // as given: NULL is HIP's null stream
    if ((rc = fut_reserve(f, fut_grid(nrep), tfut))) return rc;
    // the look-back overflow flag is sticky: mdp_future_check reads and
    // clears it, so one check covers every launch since the previous check
    return fut_launch(f, seed, rep0, nrep, tfut, (unsigned long long *)d_counts, st, true, f->derr);
}

int mdp_future_check(mdp_future *f, void *stream)
{
    if (!f) return mdp_set_error(MDP_EINVAL, "null future engine");
    FUT_TRY(hipSetDevice(f->device));
    hipStream_t st = (hipStream_t)stream;
    uint32_t err = 0;
    FUT_TRY(hipMemcpyAsync(&err, f->derr, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    FUT_TRY(hipMemsetAsync(f->derr, 0, sizeof(uint32_t), st));
    FUT_TRY(hipStreamSynchronize(st));
    if (err)
        return mdp_set_error(MDP_EUNSUPPORTED,
                             "a posterior draw needed more than %u look-back replicates (posterior mass far "
                             "below the (necstep-1)^2 scale): the device counts are not valid",
                             kLookBack);
    return MDP_OK;
}

int mdp_future_simulate(mdp_future *f, uint64_t seed, uint64_t rep0, uint64_t nrep, uint32_t tfut,
                        uint64_t *counts)
{
    int rc = fut_check_args(f, nrep, tfut);
    if (rc) return rc;
    if (!counts) return mdp_set_error(MDP_EINVAL, "null counts");
    FUT_TRY(hipSetDevice(f->device));
    if ((rc = fut_reserve(f, fut_grid(nrep), tfut))) return rc;
    if (nrep == 0) return MDP_OK;
    FUT_TRY(hipMemsetAsync(f->derr + 1, 0, sizeof(uint32_t), f->stream));
    if ((rc = fut_launch(f, seed, rep0, nrep, tfut, f->dcounts, f->stream, true, f->derr + 1))) return rc;
    std::vector<unsigned long long> h(tfut);
    uint32_t err = 0;
    FUT_TRY(hipMemcpyAsync(h.data(), f->dcounts, tfut * sizeof(unsigned long long), hipMemcpyDeviceToHost, f->stream));
    FUT_TRY(hipMemcpyAsync(&err, f->derr + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, f->stream));
    FUT_TRY(hipStreamSynchronize(f->stream));
    if (err)
        return mdp_set_error(MDP_EUNSUPPORTED,
                             "a posterior draw needed more than %u look-back replicates (posterior mass far "
                             "below the (necstep-1)^2 scale)",
                             kLookBack);
    for (uint32_t t = 0; t < tfut; ++t) counts[t] += h[t];
    return MDP_OK;
}

int mdp_future_time_kernel(mdp_future *f, uint64_t seed, uint64_t nrep, uint32_t tfut, int reps, double *ms)
{
    int rc = fut_check_args(f, nrep, tfut);
    if (rc) return rc;
    if (!ms || reps <= 0 || nrep == 0) return mdp_set_error(MDP_EINVAL, "bad timing request");
    FUT_TRY(hipSetDevice(f->device));
    if ((rc = fut_reserve(f, fut_grid(nrep), tfut))) return rc;
    if ((rc = fut_launch(f, seed, 0, nrep, tfut, f->dcounts, f->stream, false, f->derr + 1))) return rc;
    FUT_TRY(hipEventRecord(f->ev0, f->stream));
    for (int i = 0; i < reps; ++i)
        if ((rc = fut_launch(f, seed, 0, nrep, tfut, f->dcounts, f->stream, false, f->derr + 1))) return rc;
    FUT_TRY(hipEventRecord(f->ev1, f->stream));
    FUT_TRY(hipEventSynchronize(f->ev1));
    float t = 0;
    FUT_TRY(hipEventElapsedTime(&t, f->ev0, f->ev1));
    *ms = (double)t / reps;
    return MDP_OK;
}

int mdp_future_philox(uint64_t key, const uint32_t *ctr, uint32_t *out)
{
    // host restatement of the device generator, for known-answer tests of the
    // stream definition (the device path is checked through the counts)
    if (!ctr || !out) return mdp_set_error(MDP_EINVAL, "null pointer");
    uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
    uint32_t x = ctr[0], y = ctr[1], z = ctr[2], w = ctr[3];
    for (int i = 0; i < 10; ++i) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * x, p1 = (uint64_t)0xCD9E8D57u * z;
        const uint32_t nx = (uint32_t)(p1 >> 32) ^ y ^ k0, ny = (uint32_t)p1;
        const uint32_t nz = (uint32_t)(p0 >> 32) ^ w ^ k1, nw = (uint32_t)p0;
        x = nx, y = ny, z = nz, w = nw;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = x, out[1] = y, out[2] = z, out[3] = w;
    return MDP_OK;
}

}  // extern "C"
