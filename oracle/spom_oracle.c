/*
 * oracle/spom_oracle.c -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * CPU restatement of the reference MIDASPOM posterior-grid likelihood
 * (nalcala/MIDASPOM, sources/main_MIDASPOM.c), written from SURVEY.md
 * Appendix A.  It reproduces the reference's *dense* formulation and its
 * floating-point operation order (so that, with the naive row-major dgemm
 * below, the posterior file is byte-identical to the reference built
 * against a naive CBLAS -- pinned by the md5 recorded in SURVEY.md
 * Appendix C, see tests/test_oracle_golden.py).
 *
 * Callers allowed: tests/, __graft_entry__.smoke(), bench.py cpu_baseline.
 *
 * Reference anchors (file:line in /root/reference/sources/main_MIDASPOM.c):
 *   parse                     :141-167   (orc_parse)
 *   variable columns, 2^nvar  :172-175   (orc_model_load)
 *   dispersal matrix M        :177-188   (orc_model_load)
 *   piall bit encoding        :198-211   (orc_model_load)
 *   per-year states, priorst  :214-255   (orc_model_load; Q1 fixed as in
 *                                          main_MIDASPOM_MPI.c:262)
 *   short-id dedup            :256-287   (orc_model_load)
 *   grid                      :312-319   (orc_grid)
 *   hot loop body             :341-392   (orc_point_loglik)
 *     colonisation pressure   :350-358
 *     compPePc                :18-50
 *     P = Pe*Pc (dgemm)       :363
 *     forward, Q3 semantics   :368-384
 *     prior-weighted sum, log :386-392
 *   normalisation             :413-425   (orc_ltot)
 *   writer                    :427-436   (orc_write_posterior)
 */
#include "spom_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* parsing (main_MIDASPOM.c:141-167, quirk Q6)                         */
/* ------------------------------------------------------------------ */
int orc_parse(const char *path, unsigned *n_out, unsigned *tmax_out, int **obs_out)
{
    FILE *f = fopen(path, "rb");
    if (!f) return ORC_EIO;
    unsigned n = 1, tmax = 0;
    int ch;
    /* n = 1 + separators on the first line; tmax = number of '\n' */
    while ((ch = fgetc(f)) != EOF) {
        if (ch == '\n') tmax++;
        if (tmax == 0 && (ch == ' ' || ch == '\t')) n++;
    }
    rewind(f);
    int *obs = (int *)calloc((size_t)tmax * n + 1, sizeof(int));
    if (!obs) { fclose(f); return ORC_ENOMEM; }
    /* tokens stream across line breaks */
    for (size_t q = 0; q < (size_t)tmax * n; q++) {
        int v = 0;
        if (fscanf(f, "%d", &v) != 1) v = 0;
        obs[q] = v;
    }
    fclose(f);
    *n_out = n; *tmax_out = tmax; *obs_out = obs;
    return 0;
}

/* ------------------------------------------------------------------ */
/* model construction                                                  */
/* ------------------------------------------------------------------ */
int orc_model_build(const int *obs, unsigned n, unsigned tmax, double m, float p,
                    double d, orc_model **out)
{
    if (n == 0 || tmax == 0) return ORC_EINVAL;
    orc_model *md = (orc_model *)calloc(1, sizeof(orc_model));
    if (!md) return ORC_ENOMEM;
    md->n = n; md->tmax = tmax;
    md->obs = (int *)malloc(sizeof(int) * (size_t)n * tmax);
    memcpy(md->obs, obs, sizeof(int) * (size_t)n * tmax);

    /* variable columns (:172-175) */
    md->isvar = (unsigned *)calloc(n, sizeof(unsigned));
    for (unsigned t = 0; t < tmax; t++)
        for (unsigned k = 0; k < n; k++)
            if (obs[(size_t)t * n + k] != 0) md->isvar[k] = 1;
    unsigned nvar = 0;
    for (unsigned k = 0; k < n; k++) nvar += md->isvar[k];
    if (nvar > 30) { orc_model_free(md); return ORC_EINVAL; }
    md->nvar = nvar;
    md->nstates = 1u << nvar;

    /* dispersal M[i][j] = exp(-a*(j-i)*d), a = 1/m, diag 0 (:177-188).
     * Evaluated as ((-a)*(double)|j-i|)*d to keep the reference's rounding. */
    double a = 1.0 / m;
    md->M = (double *)calloc((size_t)n * n, sizeof(double));
    for (unsigned i = 0; i < n; i++)
        for (unsigned j = i + 1; j < n; j++) {
            double v = exp(-a * (double)(j - i) * d);
            md->M[(size_t)i * n + j] = v;
            md->M[(size_t)j * n + i] = v;
        }

    /* weight of each column in a state id: first var column = MSB (:198-211) */
    md->colw = (unsigned *)calloc(n, sizeof(unsigned));
    {
        unsigned rank = 0;
        for (unsigned k = 0; k < n; k++)
            if (md->isvar[k]) { md->colw[k] = 1u << (nvar - 1 - rank); rank++; }
    }

    /* per-year observed states with missing-data expansion (:214-255).
     * Non-variable columns contribute nothing (the MPI build's behaviour,
     * main_MIDASPOM_MPI.c:262; the serial build's Q1 wrap is not reproduced). */
    md->np = (unsigned *)calloc(tmax, sizeof(unsigned));
    md->yoff = (unsigned *)calloc(tmax + 1, sizeof(unsigned));
    for (unsigned t = 0; t < tmax; t++) {
        unsigned miss = 0;
        for (unsigned k = 0; k < n; k++) miss += (obs[(size_t)t * n + k] == -1);
        if (miss > 24) { orc_model_free(md); return ORC_EINVAL; }
        md->np[t] = 1u << miss;
        md->yoff[t + 1] = md->yoff[t] + md->np[t];
    }
    unsigned total = md->yoff[tmax];
    unsigned *ids = (unsigned *)calloc(total, sizeof(unsigned));
    md->prior = (float *)malloc(sizeof(float) * md->np[0]);
    for (unsigned q = 0; q < md->np[0]; q++) md->prior[q] = 1;
    for (unsigned t = 0; t < tmax; t++) {
        unsigned npt = md->np[t];
        unsigned seen = 0; /* missing columns met so far in this row */
        for (unsigned k = 0; k < n; k++) {
            int o = obs[(size_t)t * n + k];
            if (o == -1) seen++;
            for (unsigned q = 0; q < npt; q++) {
                if (o > -1) {
                    ids[md->yoff[t] + q] += (unsigned)o * md->colw[k];
                } else {
                    unsigned stride = npt >> seen;       /* = np / 2^seen */
                    unsigned bit = (q / stride) % 2;
                    ids[md->yoff[t] + q] += bit * md->colw[k];
                    if (t == 0) /* float32 prior, as main_MIDASPOM.c:248-250 */
                        md->prior[q] *= bit * p + (1 - bit) * (1 - p);
                }
            }
        }
    }
    /* short ids (:256-287): year 0 gets 0..np0-1; later states reuse the
     * short id of an identical state in an EARLIER year, else a new id. */
    md->simp = (unsigned *)calloc(total, sizeof(unsigned));
    unsigned next = 0;
    for (unsigned q = 0; q < md->np[0]; q++) md->simp[q] = next++;
    for (unsigned t = 1; t < tmax; t++) {
        for (unsigned q = 0; q < md->np[t]; q++) {
            unsigned id = ids[md->yoff[t] + q];
            int found = 0;
            unsigned sid = 0;
            for (unsigned u = 0; u < t; u++)
                for (unsigned r = 0; r < md->np[u]; r++)
                    if (ids[md->yoff[u] + r] == id) { sid = md->simp[md->yoff[u] + r]; found = 1; }
            md->simp[md->yoff[t] + q] = found ? sid : next++;
        }
    }
    md->nextid = next;
    md->short2all = (unsigned *)calloc(next, sizeof(unsigned));
    for (unsigned t = 0; t < tmax; t++)
        for (unsigned q = 0; q < md->np[t]; q++)
            md->short2all[md->simp[md->yoff[t] + q]] = ids[md->yoff[t] + q];
    free(ids);

    /* piall[j][k] = bit of state j at column k (0 for non-variable columns) */
    md->piall = (unsigned char *)calloc((size_t)md->nstates * n, 1);
    for (unsigned j = 0; j < md->nstates; j++)
        for (unsigned k = 0; k < n; k++)
            md->piall[(size_t)j * n + k] = md->isvar[k] ? ((j / md->colw[k]) % 2) : 0;

    *out = md;
    return 0;
}

int orc_model_load(const char *path, double m, float p, double d, orc_model **out)
{
    unsigned n, tmax;
    int *obs;
    int rc = orc_parse(path, &n, &tmax, &obs);
    if (rc) return rc;
    rc = orc_model_build(obs, n, tmax, m, p, d, out);
    free(obs);
    return rc;
}

void orc_model_free(orc_model *md)
{
    if (!md) return;
    free(md->obs); free(md->isvar); free(md->M); free(md->colw); free(md->np);
    free(md->yoff); free(md->prior); free(md->simp); free(md->short2all); free(md->piall);
    free(md);
}

/* accessors for ctypes */
unsigned orc_model_n(const orc_model *m) { return m->n; }
unsigned orc_model_tmax(const orc_model *m) { return m->tmax; }
unsigned orc_model_nvar(const orc_model *m) { return m->nvar; }
unsigned orc_model_nstates(const orc_model *m) { return m->nstates; }
unsigned orc_model_nextid(const orc_model *m) { return m->nextid; }
unsigned orc_model_np(const orc_model *m, unsigned t) { return t < m->tmax ? m->np[t] : 0; }
unsigned orc_model_simp(const orc_model *m, unsigned t, unsigned q)
{
    return m->simp[m->yoff[t] + q];
}
unsigned orc_model_short2all(const orc_model *m, unsigned a) { return m->short2all[a]; }
double orc_model_prior(const orc_model *m, unsigned q) { return (double)m->prior[q]; }

/* ------------------------------------------------------------------ */
/* grid (main_MIDASPOM.c:120, 312-319)                                 */
/* ------------------------------------------------------------------ */
double orc_grid(unsigned s, double lo, double hi, double *g)
{
    double win = (hi - lo) / (double)(s - 1);
    for (unsigned i = 0; i + 1 < s; i++) g[i] = ((double)i) * win + lo;
    if (s) g[s - 1] = hi;
    return win;
}

/* ------------------------------------------------------------------ */
/* one grid point (main_MIDASPOM.c:346-392)                            */
/* ------------------------------------------------------------------ */
typedef struct {
    double *Pe, *Pc, *P, *pC, *vold, *vnew;
} orc_ws;

static int ws_init(orc_ws *w, const orc_model *md)
{
    size_t ns = md->nstates, ne = md->nextid;
    unsigned npmax = 1;
    for (unsigned t = 0; t < md->tmax; t++) if (md->np[t] > npmax) npmax = md->np[t];
    size_t vsz = (size_t)md->np[0] * npmax;
    w->Pe = (double *)malloc(sizeof(double) * ne * ns);
    w->Pc = (double *)malloc(sizeof(double) * ns * ne);
    w->P = (double *)malloc(sizeof(double) * ne * ne);
    w->pC = (double *)malloc(sizeof(double) * md->n);
    w->vold = (double *)malloc(sizeof(double) * vsz);
    w->vnew = (double *)malloc(sizeof(double) * vsz);
    return (w->Pe && w->Pc && w->P && w->pC && w->vold && w->vnew) ? 0 : ORC_ENOMEM;
}

static void ws_free(orc_ws *w)
{
    free(w->Pe); free(w->Pc); free(w->P); free(w->pC); free(w->vold); free(w->vnew);
}

/* naive row-major C = A(MxK) * B(KxN), ascending-k accumulation (the CBLAS
 * call sites :363 and :379 with alpha=1, beta=0).  Every C[i][j] is
 * 0.0 + A[i][0] B[0][j] + A[i][1] B[1][j] + ... in ascending k, as the
 * textbook i-j-k loop sums it; the loops run i-k-j (rows of B streamed) and
 * skip a term whose A[i][k] is exactly 0 when row k of B is finite: it adds
 * +-0.0 to a sum that started at +0.0, which changes no bit.  Pe is zero
 * outside j <= a (compPePc, :18-50), so at 2^10 hidden states this is ~20x
 * fewer terms (round 6: 1024-state years in the GPU parity tests). */
static void naive_gemm(unsigned M, unsigned N, unsigned K, const double *A, unsigned lda,
                       const double *B, unsigned ldb, double *C, unsigned ldc)
{
    unsigned char *fin = (unsigned char *)malloc(K ? K : 1);
    for (unsigned k = 0; k < K; k++) {
        unsigned char f = 1;
        for (unsigned j = 0; j < N; j++) f &= isfinite(B[(size_t)k * ldb + j]) ? 1 : 0;
        if (fin) fin[k] = f;
    }
    for (unsigned i = 0; i < M; i++) {
        double *c = C + (size_t)i * ldc;
        for (unsigned j = 0; j < N; j++) c[j] = 0.0;
        for (unsigned k = 0; k < K; k++) {
            const double a = A[(size_t)i * lda + k];
            if (a == 0.0 && fin && fin[k]) continue;
            const double *b = B + (size_t)k * ldb;
            for (unsigned j = 0; j < N; j++) c[j] += a * b[j];
        }
    }
    free(fin);
}

static double point_loglik(const orc_model *md, orc_ws *w, double e, double c)
{
    const unsigned n = md->n, ns = md->nstates, ne = md->nextid;
    memset(w->Pe, 0, sizeof(double) * ne * ns);
    memset(w->Pc, 0, sizeof(double) * ns * ne);
    const double ebar = e > 1 ? 1 : e;
    for (unsigned j = 0; j < ns; j++) {
        const unsigned char *hid = md->piall + (size_t)j * n;   /* hidden state j */
        /* colonisation pressure (:350-358) */
        for (unsigned k = 0; k < n; k++) {
            double acc = 0;
            for (unsigned l = 0; l < n; l++)
                if (l != k) acc += md->M[(size_t)l * n + k] * hid[l];
            double pc = c * acc;
            w->pC[k] = pc > 1 ? 1 : pc;
        }
        /* extinction-then-colonisation factors (compPePc, :18-50) */
        for (unsigned a = 0; a < ne; a++) {
            const unsigned char *obs_st = md->piall + (size_t)md->short2all[a] * n;
            unsigned lost = 0, kept = 0, ok = 1;
            double col = 1;
            for (unsigned k = 0; k < n; k++) {
                unsigned h = hid[k], o = obs_st[k];
                if (h && !o) { ok = 0; break; }
                lost += (1 - h) * o;
                kept += h * o;
                col *= h + (1 - h) * ((1 - o) * (1 - w->pC[k]) + o * w->pC[k]);
            }
            if (ok) {
                w->Pe[(size_t)a * ns + j] = pow(ebar, lost) * pow(1 - ebar, kept);
                w->Pc[(size_t)j * ne + a] = col;
            }
        }
    }
    naive_gemm(ne, ne, ns, w->Pe, ns, w->Pc, ne, w->P, ne);

    /* forward propagation, Q3 semantics: row 0 of Pold = ones, other rows 0.
     * With every P entry finite the zero rows stay exactly +0.0 (0 * P
     * summed from +0.0) and add +0.0 to L, so only row 0 is propagated (the
     * same bits; at 2^10 states in year 0 the full loop is 10^9 terms a year) */
    const unsigned np0 = md->np[0];
    unsigned npprev = np0;
    int pfin = 1;
    for (size_t q = 0; q < (size_t)ne * ne && pfin; q++) pfin = isfinite(w->P[q]);
    const unsigned nrows = pfin ? 1 : np0;
    memset(w->vold, 0, sizeof(double) * (size_t)np0 * np0);
    for (unsigned q = 0; q < np0; q++) w->vold[q] = 1;
    for (unsigned t = 1; t < md->tmax; t++) {
        const unsigned npt = md->np[t];
        const unsigned *sp = md->simp + md->yoff[t - 1];
        const unsigned *sc = md->simp + md->yoff[t];
        if (nrows < np0) memset(w->vnew, 0, sizeof(double) * (size_t)np0 * npt);
        for (unsigned r = 0; r < nrows; r++)
            for (unsigned l = 0; l < npt; l++) {
                double acc = 0.0;
                for (unsigned k = 0; k < npprev; k++)
                    acc += w->vold[(size_t)r * npprev + k] * w->P[(size_t)sp[k] * ne + sc[l]];
                w->vnew[(size_t)r * npt + l] = acc;
            }
        double *tmp = w->vold; w->vold = w->vnew; w->vnew = tmp;
        npprev = npt;
    }
    double L = 0;
    for (unsigned r = 0; r < np0; r++)
        for (unsigned l = 0; l < npprev; l++)
            L += w->vold[(size_t)r * npprev + l] * (double)md->prior[r];
    return log(L);
}

int orc_loglik_rows(const orc_model *md, const double *eg, const double *cg, unsigned s,
                    unsigned ie0, unsigned ie1, double *out)
{
    orc_ws w;
    if (ws_init(&w, md)) { ws_free(&w); return ORC_ENOMEM; }
    for (unsigned ie = ie0; ie < ie1; ie++)
        for (unsigned ic = 0; ic < s; ic++)
            out[(size_t)(ie - ie0) * s + ic] = point_loglik(md, &w, eg[ie], cg[ic]);
    ws_free(&w);
    return 0;
}

/* loglik at an arbitrary list of (e,c) points (used for nested sub-grids) */
int orc_loglik_points(const orc_model *md, const double *e, const double *c, size_t npts,
                      double *out)
{
    orc_ws w;
    if (ws_init(&w, md)) { ws_free(&w); return ORC_ENOMEM; }
    for (size_t q = 0; q < npts; q++) out[q] = point_loglik(md, &w, e[q], c[q]);
    ws_free(&w);
    return 0;
}

/* multi-threaded: contiguous e-row slabs, remainder rows to slab 0, like
 * main_MIDASPOM_MPI.c:361-368 */
typedef struct {
    const orc_model *md; const double *eg, *cg; unsigned s, ie0, ie1; double *out; int rc;
} slab_arg;

static void *slab_run(void *p)
{
    slab_arg *a = (slab_arg *)p;
    a->rc = orc_loglik_rows(a->md, a->eg, a->cg, a->s, a->ie0, a->ie1,
                            a->out + (size_t)a->ie0 * a->s);
    return NULL;
}

int orc_loglik_grid_mt(const orc_model *md, const double *eg, const double *cg, unsigned s,
                       unsigned nthreads, double *out)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > s) nthreads = s;
    pthread_t *th = (pthread_t *)calloc(nthreads, sizeof(pthread_t));
    slab_arg *args = (slab_arg *)calloc(nthreads, sizeof(slab_arg));
    unsigned avg = s / nthreads, rem = s % nthreads;
    for (unsigned r = 0; r < nthreads; r++) {
        args[r].md = md; args[r].eg = eg; args[r].cg = cg; args[r].s = s; args[r].out = out;
        args[r].ie0 = r == 0 ? 0 : r * avg + rem;
        args[r].ie1 = (r + 1) * avg + rem;
        pthread_create(&th[r], NULL, slab_run, &args[r]);
    }
    int rc = 0;
    for (unsigned r = 0; r < nthreads; r++) { pthread_join(th[r], NULL); if (args[r].rc) rc = args[r].rc; }
    free(th); free(args);
    return rc;
}

/* ------------------------------------------------------------------ */
/* normalisation + writer (:413-436)                                   */
/* ------------------------------------------------------------------ */
double orc_ltot(const double *lik, unsigned s, double win)
{
    double acc = 0;
    for (unsigned k = 0; k < s; k++)
        for (unsigned l = 0; l < s; l++) {
            double wgt = 1;
            if (k == 0 || k == s - 1) wgt *= 0.5;
            if (l == 0 || l == s - 1) wgt *= 0.5;
            acc += exp(lik[(size_t)k * s + l]) * wgt;
        }
    return 2 * log(win) + log(acc);
}

int orc_write_posterior(const char *path, const double *lik, unsigned s, double ltot)
{
    FILE *f = fopen(path, "wb");
    if (!f) return ORC_EIO;
    for (unsigned i = 0; i < s; i++) {
        for (unsigned j = 0; j < s; j++) fprintf(f, "%.20lf\t", exp(lik[(size_t)i * s + j] - ltot));
        fprintf(f, "\n");
    }
    fclose(f);
    return 0;
}

/* whole run: parse -> grid -> loglik -> Ltot -> posterior file.
 * Returns Ltot through *ltot_out; writes the file when out_path != NULL. */
int orc_run(const char *in_path, const char *out_path, double m, double p, double d,
            unsigned s, double lo, double hi, unsigned nthreads, double *lik_out,
            double *ltot_out)
{
    orc_model *md;
    int rc = orc_model_load(in_path, m, (float)p, d, &md);
    if (rc) return rc;
    double *g = (double *)malloc(sizeof(double) * s);
    double win = orc_grid(s, lo, hi, g);
    double *lik = lik_out ? lik_out : (double *)malloc(sizeof(double) * (size_t)s * s);
    rc = orc_loglik_grid_mt(md, g, g, s, nthreads, lik);
    double lt = orc_ltot(lik, s, win);
    if (ltot_out) *ltot_out = lt;
    if (!rc && out_path) rc = orc_write_posterior(out_path, lik, s, lt);
    if (!lik_out) free(lik);
    free(g);
    orc_model_free(md);
    return rc;
}
