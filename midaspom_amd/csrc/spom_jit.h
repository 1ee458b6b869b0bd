// midaspom_amd/csrc/spom_jit.h -- problem-specialised forward kernel (hipRTC).
#ifndef SPOM_JIT_H
#define SPOM_JIT_H
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

struct MdpJitPlan {
    std::vector<uint32_t> np;     // possible states per year
    std::vector<uint32_t> udesc;  // per forward use: Q offset | nX << 22 | nA << 27
    size_t ldQ = 0;               // per-c Q row (doubles, even), staged in LDS
    // fused variant: the kernel computes its column's Q itself (k_qrows'
    // three phases for one c value) instead of reading Q rows
    bool fused = false;
    int fused_cols = 2;  // c columns per fused workgroup (KBLOCK threads each)
    // fused variant: the workgroup has PRO times the forward's threads; the
    // extra ones share the column-table prologue and leave before the
    // forward recursion (more threads for the latency-bound prologue, fewer
    // LDS reads per FMA in the forward: its waves take EPL points a lane)
    int pro = 1;
    bool fast_log = true;  // mdp_log (prelude) instead of the library log for log L
    // register kernels: one copy of the forward per ratio form (the t-form
    // copy without g^d factors); false: one copy for both
    bool split_forms = true;
    // several columns per workgroup: each column's lanes rotated by half a
    // block (SIMD balance of the ratio forms)
    bool rot = true;
    int hack = 0;  // diag build only (MDP_JIT_HACK; results wrong): 1 = no log, no stores; 2 = no stores
    uint32_t nj = 0, nvar = 0, nitems = 0, ncoef = 0, nqi = 0;
    // column-table layout (offsets in doubles): var-column S [nj][nvar] at 0,
    // items, qstart, qitem, the Z-row series coefficients [nj][8], then
    // zs[kmax][nj] (the explicit "large" columns)
    // ... and the reversed-copy slot of every Q-row slot (u32 [ldQ], at off_rq)
    uint32_t off_it = 0, off_qs = 0, off_qi = 0, off_rq = 0, off_zc = 0, off_zs = 0;
    uint32_t kzmax = 0;    // zs rows compiled in (grids with |c| <= 1; larger ones use k_qrows)
    bool zpad = false;     // the fused image always holds kzmax zs rows (zero past kmax)
    uint32_t qmaxlen = 0;  // most items of one Q entry
    uint32_t ct_max = 0;  // largest column-table image (doubles), for the register staging
    int epl = 0;                  // grid points per lane (0: 2 unless the weight table is large)
    int kblock = 256;             // threads per column (256 or 512)
    // states of wide years (more than 16 per year): the state vector in LDS
    // (one column per lane), each year's new states accumulated in
    // registers; every year takes the general form (EPL 1)
    bool vlds = false;
    // with vlds: waves per 64 points (1, 2 or 4); with S > 1 the workgroup
    // holds S waves for each 64 points, wave group h accumulating the new
    // states l = h mod S of a year (1/S of the accumulators each, so more
    // waves per SIMD fit beside the LDS state vectors), a barrier either
    // side of the write-back
    int vsplit = 4;
    int window = 8;               // transitions per scheduling region
    bool diag = false;            // record s_memtime phase stamps (MDP_DIAG)
    bool xcd = true;              // XCD-aware block order
    bool efast = true;            // e blocks of one column group dispatched back to back (same XCD)
    int slots = 8;                // registers caching transitions that recur (0: none)
    int wpe = 0;                  // diag build only: minimum waves per SIMD asked of the compiler (0: its default)
    double flops_pt = 0;          // out: FP64 flops per grid point of the generated code
    // a chunk of a long series (main_MIDASPOM.c:371-384 has no length limit):
    // np / udesc cover years [t0, t1] of the series; a chunk that is not the
    // first reads its start vector from the scratch vscr[state][c][e], one
    // that is not the last stores its end vector there instead of the output
    bool first = true, last = true;
    // the ratio forms' pending exponent of B at the chunk's start (the whole
    // series' schedule, so a chunked run does the one-kernel run's arithmetic
    // and hands over the same unscaled states: bit-identical results)
    uint32_t e0 = 0;
    // gather staging: Ql[i] = Qrow[qidx[i]] (udesc offsets are then into
    // this chunk's own layout); empty: the whole Q row of ldQ doubles
    std::vector<uint32_t> qidx;
    size_t ldq_row = 0;           // Q row stride when gathering (the k_qrows row)
};

// Grid points per lane for a program of these uses (2, or 1 when the weight
// table is large); chunks of one series share it, as they share a scratch.
int mdp_jit_default_epl(const std::vector<uint32_t> &udesc);

// The pending exponent of B after the plan's years, starting from plan.e0
// (the next chunk's e0).
uint32_t mdp_jit_end_exp(const MdpJitPlan &plan);

// The ratio forms' algorithmic FP64 work per grid point,
// from the plan's enumeration alone (np, udesc, e0): per point of each form
// the set-up (y = 1 - x, the ratio's division, the power tables of B and g
// beyond their first powers), every distinct Q group's Horner chain once
// (2 nX), g^d once per distinct (group, d > 0) on s-form points, each
// year's state update npc (2 npp - 1), the source pre-scales (1 per source
// above the year's minimum |A|), the flushes of the deferred exponent (npc
// multiplies + the power B^E by squaring), and the end: the prior sum
// (np_last), B^final and log (1 each).
struct MdpRatioWork {
    double setup_s = 0, setup_t = 0;  // per s-form / t-form point
    double use_s = 0, use_t = 0;      // transitions, state updates, pre-scales, flushes
    double final_pt = 0;              // prior sum, final exponent, log
};
MdpRatioWork mdp_jit_ratio_work(const MdpJitPlan &plan);

// The slot of each Q-row slot in the reversed copy the t-form lanes read:
// within each group (offset, nX + 1 coefficients) slot off + k holds
// coefficient off + nX - k; slots of no group map to themselves.
std::vector<uint32_t> mdp_jit_reversed_index(const std::vector<uint32_t> &udesc, size_t ldq);

// HIP source of `mdp_fwd_jit` for this plan; sets plan.epl when it was 0.
std::string mdp_jit_forward_source(MdpJitPlan &plan);

// A kernel mdp_log_apply(x, y, n): y[i] = mdp_log(x[i]) with the forward
// kernels' own log (the prelude), for the accuracy test.
std::string mdp_jit_log_source();

// Compile (or fetch from the memory / disk cache) a gfx950 code object.
// `fresh`: skip both caches and recompile (the runtime refused a cached
// object); the new object replaces the cached one.
// Returns 0 on success; on failure `log` holds the compiler output.
int mdp_jit_compile(const std::string &src, std::vector<char> &code, std::string &log, bool fresh = false);

#endif
