/*
 * oracle/spom_future_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's forward simulation
 * /root/reference/sources/main_MIDASPOM_future.c, in the reference's own
 * loop structure (int arrays per patch, the literal M[l][k]*pitmp[l]*K sums,
 * the linear inverse-CDF scan with its goto).  Callers allowed: tests/ (the
 * checker) and bench.py's cpu_baseline leg, never the product.
 *
 * Two random streams:
 *   ORC_RNG_PHILOX  the product's addressed stream (Philox4x32-10 keyed by
 *                   the seed, counter (replicate, year, patch pair); see
 *                   midaspom_amd/csrc/spom_future.hip): per-year counts must
 *                   agree with the GPU bit for bit.  Multithreaded over
 *                   contiguous replicate chunks.
 *   ORC_RNG_GLIBC   glibc rand() after srand(seed), drawn in the reference's
 *                   order (:361 posterior, :378 initial state, :77 extinction
 *                   of occupied patches ascending, :99 colonisation of empty
 *                   patches ascending): exactly the reference's replicate
 *                   loop for that seed (the reference seeds with time(NULL),
 *                   :345).  Single thread.  The GPU is compared with it
 *                   statistically (per-year binomial bounds).
 *
 * Parity status: the reference itself cannot be built here (it links
 * cblas_dgemm, makefile:3, and the image has no CBLAS); its only published
 * output is the manual's stochastic example (Manual_linux.pdf p.6), used as
 * a consistency check.  The restatement is otherwise parity unpinned.
 *
 * Anchors (future.c):
 *   simpij                 :64-110  (orc_simpij)
 *   survey parse           :193-225 (last row of the token stream)
 *   posterior parse        :237-262
 *   M with source row      :265-277
 *   missing completions    :286-323
 *   replicate loop         :359-386
 *   output                 :402-404
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define ORC_RNG_PHILOX 0
#define ORC_RNG_GLIBC 1

/* ---------------- Philox4x32-10 (Salmon et al. 2011) ---------------- */
void orc_philox(uint32_t k0, uint32_t k1, const uint32_t in[4], uint32_t out[4])
{
    uint32_t c0 = in[0], c1 = in[1], c2 = in[2], c3 = in[3];
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0, c1 = n1, c2 = n2, c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0, out[1] = c1, out[2] = c2, out[3] = c3;
}

/* ---------------- the problem ---------------- */
typedef struct {
    int n, necstep, npstates;
    double **M;       /* [n+1][n], row n = distance to the source (:277) */
    int **pstates;    /* [npstates][n]                                   */
    double *post;     /* [necstep][necstep]                              */
    double KD, KS;
} fut_problem;

static void fut_free(fut_problem *p)
{
    if (p->M) for (int i = 0; i < p->n + 1; i++) free(p->M[i]);
    free(p->M);
    if (p->pstates) for (int k = 0; k < p->npstates; k++) free(p->pstates[k]);
    free(p->pstates);
}

static int fut_build(fut_problem *p, const int *pend, int n, const double *post, int necstep, double m, double d,
                     double KD, double KS, double dS)
{
    memset(p, 0, sizeof *p);
    p->n = n, p->necstep = necstep, p->KD = KD, p->KS = KS;
    p->post = (double *)post;
    double a = 1.0 / m;
    p->M = (double **)malloc((n + 1) * sizeof(double *));
    for (int i = 0; i < n + 1; i++) p->M[i] = (double *)malloc(n * sizeof(double));
    for (int i = 0; i < n; i++)
        for (int j = i; j < n; j++) {
            if (i == j) p->M[i][j] = 0.0;
            else {
                p->M[i][j] = exp(-a * (j - i) * d);
                p->M[j][i] = exp(-a * (j - i) * d);
            }
        }
    for (int j = 0; j < n; j++) p->M[n][j] = exp(-a * (j + 1) * dS);
    int s1 = 0;
    for (int j = 0; j < n; j++) s1 += pend[j] == -1;
    if (s1 > 30) return -1;
    p->npstates = 1 << s1;
    p->pstates = (int **)malloc(p->npstates * sizeof(int *));
    for (int k = 0; k < p->npstates; k++) p->pstates[k] = (int *)calloc(n, sizeof(int));
    s1 = 0;
    for (int j = 0; j < n; j++) {
        if (pend[j] == -1) s1++;
        for (int k = 0; k < p->npstates; k++) {
            if (pend[j] > -1) p->pstates[k][j] = pend[j];
            else {
                int st1 = p->npstates >> s1;
                p->pstates[k][j] = k / st1 % 2;
            }
        }
    }
    return 0;
}

/* ---------------- draws ---------------- */
typedef struct {
    int mode;
    uint32_t k0, k1;
    uint64_t rep;   /* philox: current replicate */
} rng;

static double u_glibc(void) { return (double)rand() / (double)(RAND_MAX); }
static uint32_t w31(const rng *g, uint64_t rep, uint32_t t, uint32_t pair, int word)
{
    uint32_t c[4] = {(uint32_t)rep, (uint32_t)(rep >> 32), t, pair}, o[4];
    orc_philox(g->k0, g->k1, c, o);
    return o[word] >> 1;
}

/* simpij (:64-110): one year of extinction then colonisation; returns the
 * number of occupied patches.  Philox mode takes the extinction draw of
 * patch k from word 2*(k&1) and its colonisation draw from word 2*(k&1)+1
 * of philox(rep, t, k>>1). */
static int orc_simpij(const fut_problem *p, const int *piold, int *pinew, double e, double c, const rng *g,
                      uint32_t t)
{
    const int n = p->n;
    double K = p->KD, Ksource = p->KS;
    double E = e / K;
    int pitmp[64];
    double pp;
    if (E > 1) E = 1;
    for (int k = 0; k < n; k++) {
        if (piold[k] == 1) {
            pp = g->mode == ORC_RNG_GLIBC ? u_glibc()
                                          : (double)w31(g, g->rep, t, (uint32_t)k >> 1, 2 * (k & 1)) / (double)RAND_MAX;
            pitmp[k] = pp > E ? 1 : 0;
        } else {
            pitmp[k] = 0;
        }
    }
    double pCi[64];
    int res = 0;
    for (int k = 0; k < n; k++) {
        double s1 = 0;
        for (int l = 0; l < n; l++)
            if (l != k) s1 += p->M[l][k] * pitmp[l] * K;
        s1 += p->M[n][k] * Ksource;
        pCi[k] = c * s1;
        if (pCi[k] > 1) pCi[k] = 1;
        if (pitmp[k] == 0) {
            pp = g->mode == ORC_RNG_GLIBC
                     ? u_glibc()
                     : (double)w31(g, g->rep, t, (uint32_t)k >> 1, 2 * (k & 1) + 1) / (double)RAND_MAX;
            pinew[k] = pp < pCi[k] ? 1 : 0;
        } else {
            pinew[k] = 1;
        }
        res += pinew[k];
    }
    return res;
}

/* the inverse-CDF scan of :361-375; returns 1 and sets (ie, ic) if found */
static int orc_scan(const fut_problem *p, double pec, int *ie_out, int *ic_out)
{
    const int s = p->necstep;
    double pcum = 0;
    for (int ie = 0; ie < s; ie++)
        for (int ic = 0; ic < s; ic++) {
            double w = 1.0;
            if ((ie == 0) || (ie == s - 1)) w *= 0.5;
            if ((ic == 0) || (ic == s - 1)) w *= 0.5;
            pcum += w * p->post[ie * s + ic];
            if (pec < pcum) {
                *ie_out = ie, *ic_out = ic;
                return 1;
            }
        }
    return 0;
}

static double pec_of(const fut_problem *p, double u_num)
{
    /* :361  (necstep-1)*(necstep-1)*(double)rand()/(double)(RAND_MAX) */
    return (p->necstep - 1) * (p->necstep - 1) * u_num / (double)(RAND_MAX);
}

/* replicates [r0, r1) of the Philox stream, counts[t] += all-extinct */
static void run_philox(const fut_problem *p, uint64_t seed, uint64_t r0, uint64_t r1, unsigned tfut,
                       uint64_t *counts)
{
    rng g = {ORC_RNG_PHILOX, (uint32_t)seed, (uint32_t)(seed >> 32), 0};
    int n = p->n, ie, ic;
    double etmp = 0, ctmp = 0;
    /* carry-in: the (e, c) the sequential loop holds when it reaches r0 */
    for (uint64_t q = r0; q-- > 0;) {
        if (orc_scan(p, pec_of(p, (double)w31(&g, q, 0xffffffffu, 0, 0)), &ie, &ic)) {
            etmp = ie * 0.01, ctmp = ic * 0.01;
            break;
        }
    }
    int pcur[64], ptmp[64];
    for (uint64_t i = r0; i < r1; i++) {
        g.rep = i;
        if (orc_scan(p, pec_of(p, (double)w31(&g, i, 0xffffffffu, 0, 0)), &ie, &ic)) {
            etmp = ie * 0.01;
            ctmp = ic * 0.01;
        }
        int init = (int)(w31(&g, i, 0xffffffffu, 0, 1) % (uint32_t)p->npstates);
        memcpy(pcur, p->pstates[init], sizeof(int) * n);
        for (unsigned t = 0; t < tfut; t++) {
            int j = orc_simpij(p, pcur, ptmp, etmp, ctmp, &g, t);
            if (j == 0) counts[t] += 1;
            memcpy(pcur, ptmp, sizeof(int) * n);
        }
    }
}

typedef struct {
    const fut_problem *p;
    uint64_t seed, r0, r1;
    unsigned tfut;
    uint64_t *counts;
} job;

static void *job_main(void *arg)
{
    job *j = (job *)arg;
    run_philox(j->p, j->seed, j->r0, j->r1, j->tfut, j->counts);
    return NULL;
}

/* counts[t] (+=) over replicates [rep0, rep0+nrep).  mode ORC_RNG_GLIBC
 * ignores rep0 and nthreads (one sequential stream from srand(seed)). */
int orc_future_sim(const int *pend, unsigned n, const double *post, unsigned necstep, double m, double d, double KD,
                   double KS, double dS, int mode, uint64_t seed, uint64_t rep0, uint64_t nrep, unsigned tfut,
                   unsigned nthreads, uint64_t *counts)
{
    if (n == 0 || n > 64) return -1;
    fut_problem p;
    if (fut_build(&p, pend, (int)n, post, (int)necstep, m, d, KD, KS, dS)) {
        fut_free(&p);
        return -1;
    }
    if (mode == ORC_RNG_GLIBC) {
        rng g = {ORC_RNG_GLIBC, 0, 0, 0};
        int pcur[64], ptmp[64], ie, ic;
        double etmp = 0, ctmp = 0;
        srand((unsigned)seed);
        for (uint64_t i = 0; i < nrep; i++) {
            double pec = pec_of(&p, (double)rand());
            if (orc_scan(&p, pec, &ie, &ic)) {
                etmp = ie * 0.01;
                ctmp = ic * 0.01;
            }
            int init = rand() % p.npstates;
            memcpy(pcur, p.pstates[init], sizeof(int) * n);
            for (unsigned t = 0; t < tfut; t++) {
                int j = orc_simpij(&p, pcur, ptmp, etmp, ctmp, &g, t);
                if (j == 0) counts[t] += 1;
                memcpy(pcur, ptmp, sizeof(int) * n);
            }
        }
    } else {
        if (nthreads < 1) nthreads = 1;
        if (nthreads > 256) nthreads = 256;
        pthread_t th[256];
        job jobs[256];
        uint64_t *part = (uint64_t *)calloc((size_t)nthreads * (tfut ? tfut : 1), sizeof(uint64_t));
        for (unsigned k = 0; k < nthreads; k++) {
            jobs[k] = (job){&p, seed, rep0 + nrep * k / nthreads, rep0 + nrep * (k + 1) / nthreads, tfut,
                            part + (size_t)k * tfut};
            pthread_create(&th[k], NULL, job_main, &jobs[k]);
        }
        for (unsigned k = 0; k < nthreads; k++) {
            pthread_join(th[k], NULL);
            for (unsigned t = 0; t < tfut; t++) counts[t] += part[(size_t)k * tfut + t];
        }
        free(part);
    }
    fut_free(&p);
    return 0;
}
