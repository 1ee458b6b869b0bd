/*
 * include/midaspom.h -- C ABI of the MI355X-native MIDASPOM posterior-grid engine.
 *
 * The reference (nalcala/MIDASPOM) is one monolithic main() per program with
 * no library API; these entry points are the seams a C caller of the
 * reference's pipeline would bind.  Each declaration cites
 * the region of /root/reference/sources/main_MIDASPOM.c it replaces.
 *
 * Conventions
 *  - plain pointers and sizes only; no torch / HIP types in signatures
 *    (streams are passed as void*, i.e. a hipStream_t; it is used exactly as
 *    given, so NULL is HIP's null stream -- the stream torch's default
 *    `torch.cuda.current_stream().cuda_stream == 0` names);
 *  - every int-returning function returns MDP_OK (0) or a negative MDP_E*
 *    code; the reason is in mdp_last_error() (thread-local).  Nothing aborts
 *    or exits across the ABI;
 *  - an engine is not re-entrant; one host thread drives all its devices;
 *  - results are deterministic (no floating-point atomics in any reduction;
 *    the future engine's integer counts use LDS atomics, exact in any order).
 */
#ifndef MIDASPOM_H
#define MIDASPOM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MDP_OK 0
#define MDP_EINVAL (-1)       /* bad argument / malformed problem          */
#define MDP_EIO (-2)          /* cannot open / write a file                */
#define MDP_ENOMEM (-3)       /* host or device allocation failed          */
#define MDP_EHIP (-4)         /* HIP runtime error                         */
#define MDP_ENODEV (-5)       /* no usable GPU                             */
#define MDP_EUNSUPPORTED (-6) /* problem outside the engine's limits       */

#define MDP_ABI_VERSION 9

/* ------------------------------------------------------------------ */
/* Host model: parse + state enumeration (the reference's L2 layer)    */
/* ------------------------------------------------------------------ */

/* Parsed and enumerated observation model (opaque, host memory). */
typedef struct mdp_model mdp_model;

/* Read an occupancy file and enumerate its states.
 * Replaces main_MIDASPOM.c:137-287 (parse :141-167 with quirk Q6, variable
 * columns :172-175, dispersal M :177-188, state bits :198-211, per-year
 * observed states + float32 prior :214-255, short-id dedup :256-287).
 * m = mean dispersal distance (-m), p = prior occupancy of missing year-0
 * patches (-p, used as float32 like :66), d = segment length (-d). */
int mdp_model_load(const char *path, double m, float p, double d, mdp_model **out);

/* Same, from an in-memory observation matrix obs[tmax][n] (values -1/0/1). */
int mdp_model_from_obs(const int32_t *obs, uint32_t n, uint32_t tmax, double m, float p,
                       double d, mdp_model **out);

void mdp_model_free(mdp_model *model);

/* Read-only view of a model; pointers stay owned by the model. */
typedef struct mdp_problem {
    uint32_t n;                 /* patches (columns)                                 */
    uint32_t tmax;              /* years (rows)                                      */
    uint32_t nvar;              /* columns ever non-zero; nstates = 2^nvar           */
    uint32_t nextid;            /* distinct observed states ("short ids")            */
    const int32_t *obs;         /* [tmax][n] parsed observations                     */
    const uint32_t *var_cols;   /* [nvar] ascending column indices                   */
    const double *M;            /* [n][n] dispersal kernel, row-major, diag 0        */
    const uint32_t *short_state;/* [nextid] state id (first var column = MSB)        */
    const uint32_t *year_off;   /* [tmax+1] offsets into year_ids                    */
    const uint32_t *year_ids;   /* [year_off[tmax]] short ids of each year's states  */
    const float *prior;         /* [year_off[1]] float32 prior of year-0 states      */
} mdp_problem;

int mdp_model_problem(const mdp_model *model, mdp_problem *view);

/* ------------------------------------------------------------------ */
/* Grid, normalisation and posterior writer (the reference's L3/L5)    */
/* ------------------------------------------------------------------ */

/* g[i] = i*win + lo for i < s-1, g[s-1] = hi; returns win = (hi-lo)/(s-1).
 * Replaces main_MIDASPOM.c:120 and :312-319. */
double mdp_grid(uint32_t s, double lo, double hi, double *g);

/* Ltot = 2 log(win) + log(sum_k sum_l w_k w_l exp(loglik[k][l])), trapezoid
 * weights 1/2 at the grid ends.  Replaces main_MIDASPOM.c:413-425. */
double mdp_log_total(const double *loglik, uint32_t s, double win);
/* Same on any s x s view: log L of (e row k, c column l) at loglik[k*se +
 * l*sc] -- (s, 1) is the reference's lik[k][l], (1, s) the [c][e] layout the
 * device engine writes fastest (MDP_LAYOUT_CE).  Same summation order, so the
 * same bits (ABI 7). */
double mdp_log_total_view(const double *loglik, uint32_t s, size_t se, size_t sc, double win);

/* Posterior text file: "%.20lf\t" of exp(loglik-ltot) per cell, "\n" per row
 * (rows = e, columns = c).  Replaces main_MIDASPOM.c:427-436.  raw != 0
 * writes loglik itself (the MPI build's Ltot == 0 branch,
 * main_MIDASPOM_MPI.c:527). */
int mdp_write_posterior(const char *path, const double *loglik, uint32_t s, double ltot,
                        int raw);
/* Same on the view loglik[i*se + j*sc] (row i = e, column j = c); the bytes
 * written are the same as for the row-major matrix (ABI 7).  Memory held
 * while writing is bounded (a few MB per host thread) whatever s is. */
int mdp_write_posterior_view(const char *path, const double *loglik, uint32_t s, size_t se, size_t sc, double ltot,
                             int raw);

/* ------------------------------------------------------------------ */
/* GPU likelihood engine (the reference's hot loop, L3 + L4 + L6)      */
/* ------------------------------------------------------------------ */

typedef struct mdp_engine mdp_engine;

/* Build the engine on n_devices GPUs (devices == NULL -> 0..n_devices-1;
 * n_devices == 0 -> the calling thread's current HIP device).  Copies the
 * problem tables to device memory it owns and precomputes the grid-invariant
 * colonisation sums.  Replaces the setup half of main_MIDASPOM.c:341-360
 * (per-point recomputation of S = piall*M moves here, once). */
int mdp_engine_create(const mdp_problem *problem, const int *devices, int n_devices,
                      mdp_engine **out);

/* Same with engine options (ABI 7): "NAME=VALUE" pairs separated by ';', ','
 * or white space, selecting among the engine's parity-tested kernel variants
 * (MDP_FUSED=0|1, MDP_WIDE=1, MDP_JIT_CHUNK=<uses>, ...).
 * The library reads no tuning knob from the environment; mdp_engine_create
 * is this call with options == NULL (the measured defaults).  Measurement-only
 * options (MDP_DIAG, MDP_JIT_HACK, MDP_JIT_WPE) exist only in the diag build
 * (libmidaspom_diag.so, -DMDP_DIAG_BUILD); elsewhere they, like any unknown
 * name, return MDP_EINVAL. */
int mdp_engine_create_opts(const mdp_problem *problem, const int *devices, int n_devices,
                           const char *options, mdp_engine **out);

void mdp_engine_destroy(mdp_engine *engine);

/* out[ie*nc + ic] = log L(e[ie], c[ic]) (-inf where L == 0), host memory.
 * Rows are split over the engine's devices in contiguous slabs (remainder to
 * device 0, as main_MIDASPOM_MPI.c:361-368).  Replaces main_MIDASPOM.c:341-395
 * (and the MPI gather :482-506).  Every c must be finite and >= 0
 * (MDP_EINVAL otherwise, here and in mdp_engine_set_grid): the reference's
 * pC = min(1, c S) (:350-358) is a probability only there, and the kernels'
 * item factors |n - pC| and minNum clamps assume it. */
int mdp_loglik_grid(mdp_engine *engine, const double *e, uint32_t ne, const double *c,
                    uint32_t nc, double *out);

/* Device-resident variant for single-device engines (one process per GPU):
 * upload the grid once, then compute into caller-owned device memory
 * d_out[ie*ld_out + ic] on `stream` (hipStream_t; NULL = HIP's null stream).
 * mdp_engine_run is asynchronous w.r.t. the host.
 * mdp_engine_set_layout (ABI 6) selects the layout mdp_engine_run writes:
 * MDP_LAYOUT_EC (default) d_out[ie*ld_out + ic], the reference's lik[i][j]
 * (main_MIDASPOM.c:390); MDP_LAYOUT_CE d_out[ic*ld_out + ie] (ld_out >= ne),
 * where each workgroup's e values of one c column are contiguous, so its
 * stores coalesce.  Same kernels and values; mdp_loglik_grid is always EC. */
#define MDP_LAYOUT_EC 0
#define MDP_LAYOUT_CE 1
int mdp_engine_set_layout(mdp_engine *engine, int layout);
/* mdp_loglik_grid with the host result in either layout (ABI 7): EC
 * out[ie*nc + ic] (= mdp_loglik_grid), or CE out[ic*ne + ie] -- what every
 * device slab holds natively; mdp_log_total_view / mdp_write_posterior_view
 * read it in place (se = 1, sc = ne), so the drop-in CLIs never transpose. */
int mdp_loglik_grid_layout(mdp_engine *engine, const double *e, uint32_t ne, const double *c, uint32_t nc,
                           int layout, double *out);
int mdp_engine_set_grid(mdp_engine *engine, const double *e, uint32_t ne, const double *c,
                        uint32_t nc);
/* The bound the per-c tables of the following grids are built for (ABI 9):
 * max(|c| over the grid, cbound).  The Z rows split their always-zero
 * columns into explicit factors and a log series by |c| S, so
 * two grids with different max |c| evaluate some columns in different (equally
 * exact, ~1e-15) forms.  Ranks that compute column slabs of ONE grid pass
 * that grid's max |c| here, so each computes the bits a single-rank run
 * would (midaspom_amd/dist.py).  0 (the default) uses the grid's own. */
int mdp_engine_set_cbound(mdp_engine *engine, double cbound);
int mdp_engine_run(mdp_engine *engine, double *d_out, uint32_t ld_out, void *stream);

/* Kernel timing: when enabled, every kernel of a run is launched with its own
 * start/stop events (stamped from the dispatch, no extra packets on the
 * stream).  mdp_engine_kernel_ms fills up to max_k mean durations (ms) over
 * the runs since the previous call, in launch order, and returns the count;
 * mdp_engine_kernel_name gives the slot's kernel ("" for a slot the engine's
 * path does not launch: the direct path runs k_qrows + k_forward, the
 * generic path k_zpv + k_coefs + k_forward). */
int mdp_engine_set_profiling(mdp_engine *engine, int enable);
int mdp_engine_kernel_ms(mdp_engine *engine, double *ms, int max_k);
const char *mdp_engine_kernel_name(const mdp_engine *engine, int k);

/* Per-kernel durations without per-launch events: one full run into d_out,
 * then each kernel of the path launched `reps` times back to back between two
 * events on `stream`; ms[k] = mean duration of slot k (0 where the path has no
 * such kernel; names via mdp_engine_kernel_name), and a final full run leaves
 * d_out as mdp_engine_run computes it.  Returns the number of slots filled. */
int mdp_engine_time_kernels(mdp_engine *engine, double *d_out, uint32_t ld_out, void *stream, int reps,
                            double *ms, int max_k);

/* Diagnostics (diag build, option MDP_DIAG=1 at engine creation): text
 * report of per-workgroup s_memtime phase durations (shader cycles) of the
 * last run's kernels; returns the report length (0 when disabled). */
int mdp_engine_diag_report(mdp_engine *engine, char *buf, size_t len);

/* Work accounting of one run on a grid of ne x nc points (host arithmetic on
 * the enumerated problem): flops of the forward kernel in
 * the implemented factorised form, and the SURVEY.md §8(d) dense-form F_alg. */
int mdp_engine_work(const mdp_engine *engine, uint64_t ne, uint64_t nc, double *flop_impl,
                    double *flop_survey, double *bytes_min);

/* Closed-form FP64 work of the factorised algorithm on an ne x nc grid
 * (DESIGN.md §5), computed from the plan's dimensions alone -- not from any
 * kernel's emitted code -- so a roofline fraction can be recomputed from the
 * problem and a kernel duration.  Per c value: Z rows (3 flops per explicit
 * always-zero column and 2*8 + 2 for the series over the small ones, for the
 * engine's current grid), var-column pressures
 * (1 per row and var column), item factors (1 - pC where B_b = 0, one
 * multiply per free column), Q sums (len - 1 adds per entry).
 *
 * Per grid point, the algorithmic minimum of the ratio forms the forward
 * kernels evaluate (ABI 8): setup_pt -- y = 1 - x, the
 * ratio's division, the power tables past their first powers (g's on s-form
 * points only); use_pt_ratio -- every distinct Q group's Horner chain once
 * (2 nX), g^d once per distinct (group, d > 0) on s-form points, each
 * year's state update npc (2 npp - 1), the source pre-scales, the
 * deferred-exponent flushes; final_pt_ratio -- the prior sum (np_last), the
 * final B^E, log.  Those three are means over the engine's current e grid
 * (its s-form share; one half before a grid is set); pt_min is their sum and
 * flop_min = nc * per-c + ne * nc * pt_min.
 *
 * Legacy (rounds 1-4, the direct form P = sum_m Q[m] W[|A|][m] with a
 * per-point weight table, which the ratio forms no longer build):
 * weight_pt (2 maxA powers + one product per W entry used), use_pt (every
 * use 2 nX + 3), use_pt_min (each distinct transition's dot product once,
 * 2 nX + 1, plus the state updates), final_pt (2 np_last - 1); flop =
 * nc * per-c + ne * nc * (weight_pt + use_pt + final_pt) and
 * flop_min_direct the same with use_pt_min.  The per-c terms are zero on
 * the generic path (MDP_JIT=0), which has no direct plan. */
typedef struct mdp_work {
    double z_c, pc_c, item_c, q_c;        /* per c value */
    double weight_pt, use_pt, final_pt;   /* per grid point (legacy direct form) */
    double flop;                          /* the grid's total, every use (legacy) */
    double use_pt_min;                    /* per grid point, distinct transitions once (legacy) */
    double flop_min;                      /* the grid's algorithmic minimum (ratio forms, ABI 8) */
    double setup_pt, use_pt_ratio, final_pt_ratio, pt_min;  /* per grid point, ratio forms (ABI 8) */
    double flop_min_direct;               /* legacy: the direct form's minimum (flop_min before ABI 8) */
} mdp_work;
int mdp_engine_work_fact(const mdp_engine *engine, uint64_t ne, uint64_t nc, mdp_work *work);

/* Engine facts: number of devices, distinct transition pairs, forward
 * "uses" (one per consecutive-year state pair), coefficients per c value,
 * max states per year, selected kernel variant. */
typedef struct mdp_engine_info {
    int n_devices;
    uint32_t npairs;
    uint32_t nuses;
    uint32_t ncoef;
    uint32_t npmax;
    uint32_t variant;
} mdp_engine_info;
int mdp_engine_get_info(const mdp_engine *engine, mdp_engine_info *info);

/* The kernel instantiations this engine has launched so far, space-separated
 * and sorted (e.g. "k_qrows<16,0,2> mdp_fwd_jit<reading,maxA12>"): which
 * template of each hot-path kernel ran, for tests and profiles.  Writes at
 * most len bytes (NUL-terminated) and returns the full length. */
int mdp_engine_launched(const mdp_engine *engine, char *buf, size_t len);

/* y[i] = log(x[i]) on the current device with the forward kernels' own FP64
 * log (a range reduction and an atanh series; the hipRTC kernels use it for
 * log L), for its accuracy test against the host's libm. */
int mdp_log_check(const double *x, double *y, size_t n);

/* ------------------------------------------------------------------ */
/* Scenario likelihoods: in-situ die-off and habitat loss              */
/* (main_MIDASPOM_dieoff.c / main_MIDASPOM_loss.c)     */
/* ------------------------------------------------------------------ */

/* K grid, log10-spaced on [lo, hi] (dieoff.c:284-286, loss.c:315-317);
 * source-distance grid, linear on [lo, hi] (loss.c:319-322).  Return g[0]. */
double mdp_kgrid(uint32_t s, double lo, double hi, double *K);
double mdp_dgrid(uint32_t s, double lo, double hi, double *d);

typedef struct mdp_scenario mdp_scenario;

/* Engine for the likelihood of the FIRST survey row `row` (n patches, values
 * -1/0/1; dieoff.c:185-232) under the die-off (kind 0) or habitat-loss
 * (kind 1) scenario, on HIP device `device`.  m, p, d as for mdp_model_load
 * (-m, -p, -d).  n <= 16: n <= 8 runs the LDS-resident kernel (factorised
 * Pc tables in LDS), larger n a kernel whose state vectors live in HBM. */
int mdp_scenario_create(const int32_t *row, uint32_t n, double m, float p, double d, int kind, int device,
                        mdp_scenario **out);
/* Same with options (ABI 7): "MDP_SCN_BIG=1" / "MDP_SCN_ROW=1" force the
 * HBM-state / row-parallel kernel for any n they support (tests). */
int mdp_scenario_create_opts(const int32_t *row, uint32_t n, double m, float p, double d, int kind, int device,
                             const char *options, mdp_scenario **out);
void mdp_scenario_destroy(mdp_scenario *scenario);

/* out[((ie*nc + ic)*nK + iK)*nd + id] = L(e, c, K[, dsrc]) =
 * sum_i sum_s [PK^ts P^tdis]_{i,s} prior_s  (not normalised, not log), with
 * ts years before the event (-b) and tdis after (-a).  Die-off
 * (dieoff.c:304-351): PK = Pe(e/K) Pc(c K); dsrc ignored (nd = 1).  Loss
 * (loss.c:341-386): PK = Pe(e) Pc(c, source K at distance dsrc).  The
 * reference programs are the cases ne = nc = 1 (K column, or K x d table);
 * the engine evaluates any (e, c, K[, d]) product grid.  Host memory. */
int mdp_scenario_lik(mdp_scenario *scenario, int ts, int tdis, const double *e, uint32_t ne,
                     const double *c, uint32_t nc, const double *K, uint32_t nK, const double *dsrc,
                     uint32_t nd, double *out);

/* ------------------------------------------------------------------ */
/* Forward simulation of extinction under management scenarios         */
/* (main_MIDASPOM_future.c)                      */
/* ------------------------------------------------------------------ */

/* Input readers of the future program.  *row = the LAST survey row of an
 * occupancy file (n from line 1, tokens streamed across lines;
 * future.c:193-225); *post = the necstep x necstep posterior matrix, necstep
 * = separators on its first line (future.c:237-262).  Free with mdp_free. */
int mdp_future_read_survey(const char *path, uint32_t *n, uint32_t *tmax, int32_t **row);
int mdp_future_read_posterior(const char *path, uint32_t *necstep, double **post);
void mdp_free(void *p);

typedef struct mdp_future mdp_future;

/* Engine for the replicate loop of future.c:343-386 on HIP device `device`:
 * last survey row (n <= 64 patches, values -1/0/1, <= 30 missing), the
 * posterior it samples (e, c) from (row-major necstep^2; e = ie*0.01 and
 * c = ic*0.01 as hard-coded at :370-371), m = mean dispersal (-m), d =
 * segment length (-d), KD = relative population size (-D), KS = source
 * size (-S), dS = source distance (-s). */
int mdp_future_create(const int32_t *last_row, uint32_t n, const double *post, uint32_t necstep, double m,
                      double d, double KD, double KS, double dS, int device, mdp_future **out);
void mdp_future_destroy(mdp_future *future);

/* counts[t] += number of replicates r in [rep0, rep0 + nrep) with every patch
 * empty after year t+1, t < tfut (future.c:381-385; Lik[] there).  Draws are
 * Philox4x32-10 keyed by `seed` and addressed by (replicate, year, patch):
 * results do not depend on how replicates are split (over GPUs, ranks or
 * calls).  Host memory. */
int mdp_future_simulate(mdp_future *future, uint64_t seed, uint64_t rep0, uint64_t nrep, uint32_t tfut,
                        uint64_t *counts);
/* Same into caller-owned device memory d_counts[tfut] (overwritten, not
 * accumulated) on `stream` (NULL = HIP's null stream); asynchronous.  A
 * replicate whose posterior draw needs more look-back than the engine holds
 * raises a sticky device error flag; mdp_future_check waits for `stream`,
 * reads and clears the flag, and returns MDP_EUNSUPPORTED when it was set --
 * the counts of some launch since the previous check are then not valid, so
 * one check after several launches covers all of them (the host form
 * mdp_future_simulate checks its own launch with a separate flag). */
int mdp_future_simulate_device(mdp_future *future, uint64_t seed, uint64_t rep0, uint64_t nrep, uint32_t tfut,
                               uint64_t *d_counts, void *stream);
int mdp_future_check(mdp_future *future, void *stream);
/* Mean duration (ms) of the simulation kernel over `reps` back-to-back
 * launches of replicates [0, nrep) between two events. */
int mdp_future_time_kernel(mdp_future *future, uint64_t seed, uint64_t nrep, uint32_t tfut, int reps, double *ms);
/* The generator itself: out[4] = Philox4x32-10(key, ctr[4]) (host). */
int mdp_future_philox(uint64_t key, const uint32_t *ctr, uint32_t *out);

/* Device-resident form of mdp_scenario_lik (one process per GPU): upload the
 * grid once (set_grid; ts, tdis and the axes as above), then compute into
 * caller-owned device memory d_out[ne*nc*nK*nd] (same layout) on `stream`
 * (NULL = HIP's null stream), asynchronously.  time_kernels: ms[0] =
 * mean duration of the v = P^tdis w kernel, ms[1] = of the PK^ts kernel,
 * each launched `reps` times back to back between two events. */
int mdp_scenario_set_grid(mdp_scenario *scenario, int ts, int tdis, const double *e, uint32_t ne, const double *c,
                          uint32_t nc, const double *K, uint32_t nK, const double *dsrc, uint32_t nd);
int mdp_scenario_run(mdp_scenario *scenario, double *d_out, void *stream);
int mdp_scenario_time_kernels(mdp_scenario *scenario, double *d_out, void *stream, int reps, double *ms);

/* Thread-local description of the last error. */
const char *mdp_last_error(void);

int mdp_abi_version(void);

/* Number of visible HIP devices (0 when none); the CLIs use it to deal work
 * over GPUs. */
int mdp_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* MIDASPOM_H */
