/*
 * oracle/spom_dieoff_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's two scenario likelihoods, in the
 * reference's dense operation order (full 2^n state space, naive row-major
 * dgemm, the same binary matrix power):
 *   in-situ die-off   /root/reference/sources/main_MIDASPOM_dieoff.c
 *   habitat loss      /root/reference/sources/main_MIDASPOM_loss.c
 * Callers allowed: tests/ (checker), never the product.
 *
 * Pinned by the manual's worked examples (Manual_linux.pdf p.4 dieoff and
 * p.5 loss tables, tests/golden/anchors.json) in tests/test_oracle_golden.py.
 *
 * Anchors (dieoff.c unless noted):
 *   matpow                    :17-49   (orc_matpow)
 *   pije  (E = min(1, e/K))   :51-64   (loss.c:52-65: E = min(1, e))
 *   pijc  (pC = c*s1*K)       :66-83
 *   pijcsource (loss)         loss.c:86-105  (s1 += M[n][k]*Ksource, pC = c*s1)
 *   first survey row, states  :185-232
 *   dispersal M               :238-248 (loss.c:269-279 + source row :365)
 *   K grid (log10)            :284-286;  d grid (loss)  loss.c:319-322
 *   P = Pe*Pc, P^tdis         :307-316
 *   per K: PK, PK^ts, PK^ts*P^tdis, sum over columns of observed states
 *                             :322-351  (loss.c:360-386)
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* c = a*b, row-major n x n, the reference's cblas_dgemm(RowMajor,NoTrans,NoTrans):
 * every c[i][j] is the k-ascending sum s += a[i][k]*b[k][j].  For n > 8
 * patches (2^n >= 512 states) b is transposed first, the rows are split over
 * threads and each dot product runs as four interleaved partial sums -- a
 * reordering of the same sum, as any optimised BLAS the reference links
 * makes (naive and OpenBLAS reference outputs differ by <= 1e-13, SURVEY
 * Appendix C); n <= 8 keeps the exact k-ascending order. */
struct dg_job {
    const double *a, *bt;
    double *c;
    int n, i0, i1;
};

static void *dg_rows(void *arg)
{
    const struct dg_job *J = arg;
    const int n = J->n;
    for (int i = J->i0; i < J->i1; ++i)
        for (int j = 0; j < n; ++j) {
            const double *ar = J->a + (size_t)i * n, *br = J->bt + (size_t)j * n;
            double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;  /* n is a multiple of 4 here */
            for (int k = 0; k < n; k += 4) {
                s0 += ar[k] * br[k];
                s1 += ar[k + 1] * br[k + 1];
                s2 += ar[k + 2] * br[k + 2];
                s3 += ar[k + 3] * br[k + 3];
            }
            J->c[(size_t)i * n + j] = (s0 + s1) + (s2 + s3);
        }
    return NULL;
}

static void dgemm(const double *a, const double *b, double *c, int n)
{
    if (n <= 256) {
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) {
                double s = 0.0;
                for (int k = 0; k < n; ++k) s += a[i * n + k] * b[k * n + j];
                c[i * n + j] = s;
            }
        return;
    }
    double *bt = malloc(sizeof(double) * (size_t)n * n);
    for (int k = 0; k < n; ++k)
        for (int j = 0; j < n; ++j) bt[(size_t)j * n + k] = b[(size_t)k * n + j];
    long nt = sysconf(_SC_NPROCESSORS_ONLN);
    const char *ev = getenv("OMP_NUM_THREADS");
    if (ev && atoi(ev) > 0) nt = atoi(ev);
    if (nt > 16) nt = 16;
    if (nt < 1) nt = 1;
    pthread_t th[16];
    struct dg_job jobs[16];
    for (int t = 0; t < nt; ++t) {
        jobs[t] = (struct dg_job){a, bt, c, n, (int)((long)n * t / nt), (int)((long)n * (t + 1) / nt)};
        if (t) pthread_create(&th[t], NULL, dg_rows, &jobs[t]);
    }
    dg_rows(&jobs[0]);
    for (int t = 1; t < nt; ++t) pthread_join(th[t], NULL);
    free(bt);
}

/* z = x^k, dieoff.c:17-49 (x is overwritten, as in the reference) */
static void orc_matpow(double *x, int n, int k, double *z)
{
    if (k == 0) {
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) z[i * n + j] = i == j ? 1.0 : 0.0;
        return;
    }
    double *tmp = malloc(sizeof(double) * n * n);
    memcpy(z, x, sizeof(double) * n * n);
    k--;
    while (k > 0) {
        if (k & 1) {
            dgemm(x, z, tmp, n);
            memcpy(z, tmp, sizeof(double) * n * n);
        }
        if (k == 1) break;
        k >>= 1;
        dgemm(x, x, tmp, n);
        memcpy(x, tmp, sizeof(double) * n * n);
    }
    free(tmp);
}

static int bit(int s, int j, int n) { return (s >> (n - 1 - j)) & 1; }

/* extinction phase, dieoff.c:51-64 (K = 1 gives loss.c's pije) */
static double pije(int from, int to, double e, double K, int n)
{
    int s1 = 0, s2 = 0;
    double E = e / K;
    if (E > 1) E = 1;
    for (int k = 0; k < n; ++k) {
        const int po = bit(from, k, n), pt = bit(to, k, n);
        if (pt * (1 - po) > 0) return 0;
        s1 += (1 - pt) * po;
        s2 += pt * po;
    }
    return pow(E, s1) * pow(1 - E, s2);
}

/* colonisation phase: dieoff.c:66-83 (src == NULL) or loss.c:86-105 */
static double pijc(int tmp, int nw, double c, double K, const double *M, const double *src, double Ks, int n)
{
    double res = 1;
    for (int k = 0; k < n; ++k) {
        const int pt = bit(tmp, k, n), pn = bit(nw, k, n);
        if (pt * (1 - pn) > 0) return 0;
        double s1 = 0;
        for (int l = 0; l < n; ++l)
            if (l != k) s1 += M[l * n + k] * bit(tmp, l, n);
        double pC;
        if (src) {
            s1 += src[k] * Ks;
            pC = c * s1;
        } else {
            pC = c * s1 * K;
        }
        if (pC > 1) pC = 1;
        res *= pt + (1 - pt) * (1 - pn) * (1 - pC) + (1 - pt) * pn * pC;
    }
    return res;
}

/* first-survey states and float priors, dieoff.c:198-232 */
static int states_of(const int32_t *row, int n, float p, int **ps, float **pr)
{
    int s1 = 0;
    for (int j = 0; j < n; ++j) s1 += row[j] == -1;
    const int np = 1 << s1;
    *ps = calloc(np, sizeof(int));
    *pr = malloc(np * sizeof(float));
    for (int k = 0; k < np; ++k) (*pr)[k] = 1;
    s1 = 0;
    for (int j = 0; j < n; ++j) {
        if (row[j] == -1) s1++;
        for (int k = 0; k < np; ++k) {
            if (row[j] > -1) {
                (*ps)[k] += row[j] * (1 << (n - j - 1));
            } else {
                const int st1 = np >> s1;
                (*ps)[k] += (k / st1 % 2) * (1 << (n - j - 1));
                (*pr)[k] *= (k / st1 % 2) * p + (1 - k / st1 % 2) * (1 - p);
            }
        }
    }
    return np;
}

static void dispersal(int n, double m, double d, double *M)
{
    const double a = 1.0 / m;
    for (int i = 0; i < n; ++i)
        for (int j = i; j < n; ++j) {
            if (i == j) M[i * n + j] = 0.0;
            else M[i * n + j] = M[j * n + i] = exp(-a * (j - i) * d);
        }
}

/* log10 K grid, dieoff.c:284-286 */
void orc_kgrid(uint32_t s, double lo, double hi, double *K)
{
    for (uint32_t i = 0; i < s; ++i)
        K[i] = pow(10.0, ((double)i) / (s - 1) * (log10(hi) - log10(lo)) + log10(lo));
}

/* L = sum_i sum_j [PK^ts P^tdis]_{i, ps_j} pr_j for each K (and source
 * distance), i.e. dieoff.c:304-351 / loss.c:341-386.  out[iK * nd + id]. */
static int scenario(const int32_t *row, uint32_t n, double m, float p, double d, int ts, int tdis, double e,
                    double c, const double *K, uint32_t nK, const double *dsrc, uint32_t nd, int loss,
                    double *out)
{
    if (n == 0 || n > 12) return -1;
    const int ns = 1 << n;
    int *ps;
    float *pr;
    const int np = states_of(row, (int)n, p, &ps, &pr);
    double *M = malloc(sizeof(double) * n * n), *src = malloc(sizeof(double) * n);
    dispersal((int)n, m, d, M);
    const size_t sz = (size_t)ns * ns * sizeof(double);
    double *Pe = malloc(sz), *Pc = malloc(sz), *P = malloc(sz), *Ppow = malloc(sz), *PK = malloc(sz),
           *PKpow = malloc(sz), *Ptot = malloc(sz);
    for (int i = 0; i < ns; ++i)
        for (int j = 0; j < ns; ++j) {
            Pe[i * ns + j] = pije(i, j, e, 1.0, (int)n);
            Pc[i * ns + j] = pijc(i, j, c, 1.0, M, NULL, 0.0, (int)n);
        }
    dgemm(Pe, Pc, P, ns);
    orc_matpow(P, ns, tdis, Ppow);
    const double a = 1.0 / m;
    for (uint32_t iK = 0; iK < nK; ++iK)
        for (uint32_t id = 0; id < (loss ? nd : 1u); ++id) {
            if (loss)
                for (uint32_t j = 0; j < n; ++j) src[j] = exp(-a * (j + 1) * dsrc[id]);
            for (int i = 0; i < ns; ++i)
                for (int j = 0; j < ns; ++j) {
                    Pe[i * ns + j] = pije(i, j, e, loss ? 1.0 : K[iK], (int)n);
                    Pc[i * ns + j] = loss ? pijc(i, j, c, 1.0, M, src, K[iK], (int)n)
                                          : pijc(i, j, c, K[iK], M, NULL, 0.0, (int)n);
                }
            dgemm(Pe, Pc, PK, ns);
            orc_matpow(PK, ns, ts, PKpow);
            dgemm(PKpow, Ppow, Ptot, ns);
            double L = 0;
            for (int i = 0; i < ns; ++i)
                for (int j = 0; j < np; ++j) L += Ptot[i * ns + ps[j]] * pr[j];
            out[(size_t)iK * (loss ? nd : 1u) + id] = L;
        }
    free(Pe), free(Pc), free(P), free(Ppow), free(PK), free(PKpow), free(Ptot);
    free(M), free(src), free(ps), free(pr);
    return 0;
}

int orc_dieoff_lik(const int32_t *row, uint32_t n, double m, float p, double d, int ts, int tdis, double e,
                   double c, const double *K, uint32_t nK, double *out)
{
    return scenario(row, n, m, p, d, ts, tdis, e, c, K, nK, NULL, 0, 0, out);
}

int orc_loss_lik(const int32_t *row, uint32_t n, double m, float p, double d, int ts, int tdis, double e,
                 double c, const double *K, uint32_t nK, const double *dsrc, uint32_t nd, double *out)
{
    return scenario(row, n, m, p, d, ts, tdis, e, c, K, nK, dsrc, nd, 1, out);
}

/* The same likelihood by vector propagation, for n up to 20 patches where the
 * dense 2^n x 2^n products above are out of reach (the GPU's k_scn_big range,
 * n = 13..16).  L = 1' PK^ts P^tdis w with w[ps_j] = pr_j, applied right to
 * left: u <- Pe (Pc u) per year.  Every matrix entry is the reference's own
 * expression (pije :51-64, pijc :66-83 / loss.c:86-105, with the colonisation
 * sums s1 of a row computed once in pijc's l order), and each row's sum runs
 * over k ascending as the dense row-major product does, skipping only the
 * entries pije / pijc return as exact zeros (j not within the source state).
 * What differs from the reference is the association of the products (matrix
 * powers first there), so agreement is to rounding, not bitwise; it is
 * checked against orc_dieoff_lik / orc_loss_lik at small n
 * (tests/test_scenario_oracle.py).  out = L for one (e, c, K[, d]). */
static void scn_apply(int n, const double *M, const double *src, double Ks, int loss, double e, double c, double K,
                      const double *u, double *z, double *y)
{
    const int ns = 1 << n;
    /* z = Pc u: row j, columns nw >= j bitwise.  pijc's per-patch factor
     * pt + (1-pt)(1-pn)(1-pC) + (1-pt) pn pC takes one of two values per
     * (k, pn) for a row (pt fixed): evaluated once with the same expression */
    double fac[32][2];
    for (int j = 0; j < ns; ++j) {
        for (int k = 0; k < n; ++k) {
            double s1 = 0;
            for (int l = 0; l < n; ++l)
                if (l != k) s1 += M[l * n + k] * bit(j, l, n);
            double pc;
            if (loss) {
                s1 += src[k] * Ks;
                pc = c * s1;
            } else {
                pc = c * s1 * K;
            }
            const double pC = pc > 1 ? 1 : pc;
            const int pt = bit(j, k, n);
            for (int pn = 0; pn < 2; ++pn)
                fac[k][pn] = pt + (1 - pt) * (1 - pn) * (1 - pC) + (1 - pt) * pn * pC;
        }
        double acc = 0;
        for (int nw = j; nw < ns; nw = (nw + 1) | j) {
            double res = 1;
            for (int k = 0; k < n; ++k) res *= fac[k][bit(nw, k, n)];
            acc += res * u[nw];
        }
        z[j] = acc;
    }
    /* y = Pe z: row i, columns j <= i bitwise (ascending subsets); pije's
     * pow(E, lost) * pow(1 - E, kept) from tables of the same pow values */
    double E = loss ? e : e / K;
    if (E > 1) E = 1;
    double pe[33], pk[33];
    for (int s = 0; s <= n; ++s) {
        pe[s] = pow(E, s);
        pk[s] = pow(1 - E, s);
    }
    for (int i = 0; i < ns; ++i) {
        double acc = 0;
        for (int j = 0;; j = (j - i) & i) {
            acc += pe[__builtin_popcount(i & ~j)] * pk[__builtin_popcount(j)] * z[j];
            if (j == i) break;
        }
        y[i] = acc;
    }
}

int orc_scenario_vec(const int32_t *row, uint32_t n, double m, float p, double d, int ts, int tdis, double e,
                     double c, double K, double dsrc, int loss, double *out)
{
    if (n == 0 || n > 20) return -1;
    const int ns = 1 << n;
    int *ps;
    float *pr;
    const int np = states_of(row, (int)n, p, &ps, &pr);
    double *M = malloc(sizeof(double) * n * n), *src = malloc(sizeof(double) * n);
    dispersal((int)n, m, d, M);
    const double a = 1.0 / m;
    for (uint32_t j = 0; j < n; ++j) src[j] = exp(-a * (j + 1) * dsrc);
    double *u = calloc(ns, sizeof(double)), *z = malloc(sizeof(double) * ns), *y = malloc(sizeof(double) * ns);
    for (int j = 0; j < np; ++j) u[ps[j]] += pr[j];
    for (int t = 0; t < tdis; ++t) {  /* P = Pe Pc at K = 1, no source */
        scn_apply((int)n, M, src, 0.0, 0, e, c, 1.0, u, z, y);
        memcpy(u, y, sizeof(double) * ns);
    }
    for (int t = 0; t < ts; ++t) {    /* PK */
        scn_apply((int)n, M, src, K, loss, e, c, loss ? 1.0 : K, u, z, y);
        memcpy(u, y, sizeof(double) * ns);
    }
    double L = 0;
    for (int i = 0; i < ns; ++i) L += u[i];
    *out = L;
    free(u), free(z), free(y), free(M), free(src), free(ps), free(pr);
    return 0;
}
