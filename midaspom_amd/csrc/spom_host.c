/*
 * midaspom_amd/csrc/spom_host.c -- host side of the MIDASPOM engine:
 * occupancy-file parser, state enumeration, (e,c) grid, trapezoid
 * normalisation and the posterior writer.  These keep the reference's file
 * formats and numerics; the likelihood itself runs on
 * the GPU (spom_engine.hip).
 *
 * Reference regions (/root/reference/sources/main_MIDASPOM.c):
 *   mdp_model_load / parse_occupancy   :141-167  (n from line-1 separators,
 *                                                 tmax from '\n', tokens
 *                                                 stream across lines: Q6)
 *   build_model                        :172-287
 *   mdp_grid                           :120, :312-319
 *   mdp_log_total                      :413-425
 *   mdp_write_posterior                :427-436  (+ main_MIDASPOM_MPI.c:527)
 */
#include <math.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "mdp_internal.h"

static __thread char g_err[512];

int mdp_set_error(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

const char *mdp_last_error(void) { return g_err; }

int mdp_abi_version(void) { return MDP_ABI_VERSION; }

/* ------------------------------------------------------------------ */
/* parser                                                              */
/* ------------------------------------------------------------------ */

/* Token reader: whitespace-separated decimal integers, like fscanf("%d").
 * A token that does not parse leaves the value 0 and stops reading (the
 * reference leaves the cell uninitialised). */
static int parse_occupancy(const char *path, uint32_t *n_out, uint32_t *tmax_out, int32_t **obs_out)
{
    FILE *f = fopen(path, "rb");
    if (!f) return mdp_set_error(MDP_EIO, "cannot open input file '%s'", path);
    if (fseek(f, 0, SEEK_END) != 0) { fclose(f); return mdp_set_error(MDP_EIO, "cannot seek '%s'", path); }
    long len = ftell(f);
    rewind(f);
    char *buf = (char *)malloc((size_t)len + 1);
    if (!buf) { fclose(f); return mdp_set_error(MDP_ENOMEM, "out of host memory"); }
    size_t got = fread(buf, 1, (size_t)len, f);
    fclose(f);
    buf[got] = 0;

    uint32_t n = 1, tmax = 0;
    for (size_t q = 0; q < got; q++) {
        char ch = buf[q];
        if (ch == '\n') tmax++;
        else if (tmax == 0 && (ch == ' ' || ch == '\t')) n++;
    }
    if (tmax == 0) { free(buf); return mdp_set_error(MDP_EINVAL, "input '%s' has no complete line", path); }
    size_t cells = (size_t)tmax * n;
    int32_t *obs = (int32_t *)calloc(cells, sizeof(int32_t));
    if (!obs) { free(buf); return mdp_set_error(MDP_ENOMEM, "out of host memory"); }
    const char *p = buf;
    for (size_t q = 0; q < cells; q++) {
        char *end;
        while (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r' || *p == '\v' || *p == '\f') p++;
        if (!*p) break;
        long v = strtol(p, &end, 10);
        if (end == p) break;
        obs[q] = (int32_t)v;
        p = end;
    }
    free(buf);
    *n_out = n; *tmax_out = tmax; *obs_out = obs;
    return MDP_OK;
}

/* ------------------------------------------------------------------ */
/* state enumeration                                                   */
/* ------------------------------------------------------------------ */

/* open-addressing map: state id -> short id */
typedef struct { uint32_t *key, *val; uint32_t mask; } idmap;

static int idmap_init(idmap *m, uint32_t expected)
{
    uint32_t cap = 16;
    while (cap < 2 * expected + 1) cap <<= 1;
    m->key = (uint32_t *)malloc(sizeof(uint32_t) * cap);
    m->val = (uint32_t *)malloc(sizeof(uint32_t) * cap);
    if (!m->key || !m->val) return -1;
    memset(m->key, 0xff, sizeof(uint32_t) * cap);
    m->mask = cap - 1;
    return 0;
}

static uint32_t *idmap_slot(idmap *m, uint32_t key, int *found)
{
    uint32_t h = (key * 2654435761u) & m->mask;
    while (m->key[h] != 0xffffffffu && m->key[h] != key) h = (h + 1) & m->mask;
    *found = m->key[h] == key;
    m->key[h] = key;
    return &m->val[h];
}

int mdp_model_from_obs(const int32_t *obs, uint32_t n, uint32_t tmax, double m, float p,
                       double d, mdp_model **out)
{
    if (!obs || !out || n == 0 || tmax == 0) return mdp_set_error(MDP_EINVAL, "empty observation matrix");
    if (!(m > 0) && !(m < 0)) return mdp_set_error(MDP_EINVAL, "mean dispersal -m must be non-zero");
    mdp_model *md = (mdp_model *)calloc(1, sizeof(mdp_model));
    if (!md) return mdp_set_error(MDP_ENOMEM, "out of host memory");
    md->n = n; md->tmax = tmax;
    md->obs = (int32_t *)malloc(sizeof(int32_t) * (size_t)n * tmax);
    uint8_t *isvar = (uint8_t *)calloc(n, 1);
    int rc = MDP_OK;
    if (!md->obs || !isvar) { rc = mdp_set_error(MDP_ENOMEM, "out of host memory"); goto fail; }
    memcpy(md->obs, obs, sizeof(int32_t) * (size_t)n * tmax);
    for (size_t q = 0; q < (size_t)n * tmax; q++)
        if (obs[q] < -1 || obs[q] > 1) {
            rc = mdp_set_error(MDP_EINVAL, "observation %d at year %zu patch %zu is not -1, 0 or 1",
                               obs[q], q / n, q % n);
            goto fail;
        }

    /* a column is variable if any year is non-zero (:172-175) */
    for (size_t q = 0; q < (size_t)n * tmax; q++) if (obs[q] != 0) isvar[q % n] = 1;
    uint32_t nvar = 0;
    for (uint32_t k = 0; k < n; k++) nvar += isvar[k];
    if (nvar > 30) { rc = mdp_set_error(MDP_EUNSUPPORTED, "%u variable columns: 2^nvar hidden states exceed 32-bit ids", nvar); goto fail; }
    md->nvar = nvar;
    md->var_cols = (uint32_t *)malloc(sizeof(uint32_t) * (nvar ? nvar : 1));
    uint32_t *weight = (uint32_t *)calloc(n, sizeof(uint32_t));
    if (!md->var_cols || !weight) { free(weight); rc = mdp_set_error(MDP_ENOMEM, "out of host memory"); goto fail; }
    for (uint32_t k = 0, r = 0; k < n; k++)
        if (isvar[k]) { md->var_cols[r] = k; weight[k] = 1u << (nvar - 1 - r); r++; }

    /* dispersal kernel, evaluated as ((-1/m)*|i-j|)*d like :183-184 */
    md->M = (double *)calloc((size_t)n * n, sizeof(double));
    if (!md->M) { free(weight); rc = mdp_set_error(MDP_ENOMEM, "out of host memory"); goto fail; }
    {
        const double a = 1.0 / m;
        for (uint32_t i = 0; i < n; i++)
            for (uint32_t j = i + 1; j < n; j++) {
                const double v = exp(-a * (double)(j - i) * d);
                md->M[(size_t)i * n + j] = v;
                md->M[(size_t)j * n + i] = v;
            }
    }

    /* observed states: each -1 doubles the year's state list; the first
     * missing column is the most significant bit of the expansion index */
    md->year_off = (uint32_t *)calloc(tmax + 1, sizeof(uint32_t));
    if (!md->year_off) { free(weight); rc = mdp_set_error(MDP_ENOMEM, "out of host memory"); goto fail; }
    for (uint32_t t = 0; t < tmax; t++) {
        uint32_t miss = 0;
        for (uint32_t k = 0; k < n; k++) miss += obs[(size_t)t * n + k] == -1;
        if (miss > 20) { free(weight); rc = mdp_set_error(MDP_EUNSUPPORTED, "year %u has %u missing patches (limit 20)", t, miss); goto fail; }
        md->year_off[t + 1] = md->year_off[t] + (1u << miss);
    }
    const uint32_t total = md->year_off[tmax];
    const uint32_t np0 = md->year_off[1];
    uint32_t *state = (uint32_t *)malloc(sizeof(uint32_t) * total);
    md->year_ids = (uint32_t *)malloc(sizeof(uint32_t) * total);
    md->prior = (float *)malloc(sizeof(float) * np0);
    uint32_t *misscol = (uint32_t *)malloc(sizeof(uint32_t) * (n + 1));
    if (!state || !md->year_ids || !md->prior || !misscol) {
        free(state); free(misscol); free(weight);
        rc = mdp_set_error(MDP_ENOMEM, "out of host memory"); goto fail;
    }
    for (uint32_t t = 0; t < tmax; t++) {
        const int32_t *row = obs + (size_t)t * n;
        uint32_t base = 0, nm = 0;
        for (uint32_t k = 0; k < n; k++) {
            if (row[k] == -1) misscol[nm++] = k;
            else if (row[k] > 0) base += (uint32_t)row[k] * weight[k];
        }
        const uint32_t npt = 1u << nm;
        for (uint32_t q = 0; q < npt; q++) {
            uint32_t id = base;
            float pr = 1;
            for (uint32_t r = 0; r < nm; r++) {
                const uint32_t bit = (q >> (nm - 1 - r)) & 1u;
                id += bit * weight[misscol[r]];
                if (t == 0) pr *= bit ? p : 1.0f - p; /* float32, :248-250 */
            }
            state[md->year_off[t] + q] = id;
            if (t == 0) md->prior[q] = pr;
        }
    }
    free(misscol);
    free(weight);

    /* short ids: year 0 -> 0..np0-1; afterwards first occurrence wins */
    idmap map;
    if (idmap_init(&map, total)) { free(state); rc = mdp_set_error(MDP_ENOMEM, "out of host memory"); goto fail; }
    uint32_t next = 0;
    for (uint32_t q = 0; q < total; q++) {
        int found;
        uint32_t *slot = idmap_slot(&map, state[q], &found);
        if (!found || q < np0) *slot = next++;
        md->year_ids[q] = *slot;
    }
    md->nextid = next;
    md->short_state = (uint32_t *)malloc(sizeof(uint32_t) * next);
    if (!md->short_state) { free(map.key); free(map.val); free(state); rc = mdp_set_error(MDP_ENOMEM, "out of host memory"); goto fail; }
    for (uint32_t q = 0; q < total; q++) md->short_state[md->year_ids[q]] = state[q];
    free(map.key); free(map.val); free(state);
    free(isvar);
    *out = md;
    return MDP_OK;
fail:
    free(isvar);
    mdp_model_free(md);
    return rc;
}

int mdp_model_load(const char *path, double m, float p, double d, mdp_model **out)
{
    if (!path || !out) return mdp_set_error(MDP_EINVAL, "null argument");
    uint32_t n = 0, tmax = 0;
    int32_t *obs = NULL;
    int rc = parse_occupancy(path, &n, &tmax, &obs);
    if (rc) return rc;
    rc = mdp_model_from_obs(obs, n, tmax, m, p, d, out);
    free(obs);
    return rc;
}

void mdp_model_free(mdp_model *md)
{
    if (!md) return;
    free(md->obs); free(md->var_cols); free(md->M); free(md->short_state);
    free(md->year_off); free(md->year_ids); free(md->prior);
    free(md);
}

int mdp_model_problem(const mdp_model *md, mdp_problem *v)
{
    if (!md || !v) return mdp_set_error(MDP_EINVAL, "null argument");
    v->n = md->n; v->tmax = md->tmax; v->nvar = md->nvar; v->nextid = md->nextid;
    v->obs = md->obs; v->var_cols = md->var_cols; v->M = md->M;
    v->short_state = md->short_state; v->year_off = md->year_off;
    v->year_ids = md->year_ids; v->prior = md->prior;
    return MDP_OK;
}

/* ------------------------------------------------------------------ */
/* grid, normalisation, writer                                         */
/* ------------------------------------------------------------------ */

double mdp_grid(uint32_t s, double lo, double hi, double *g)
{
    const double win = (hi - lo) / (double)(s - 1);
    if (g && s) {
        for (uint32_t i = 0; i + 1 < s; i++) g[i] = (double)i * win + lo;
        g[s - 1] = hi;
    }
    return win;
}

/* ------------------------------------------------------------------ */
/* host threads for the per-cell work of a large grid (exp, formatting) */
/* ------------------------------------------------------------------ */

/* OMP_NUM_THREADS when set, else the online CPUs, at most 16; one thread
 * below 64 Ki cells */
static unsigned host_threads(size_t cells)
{
    if (cells < (1u << 16)) return 1;
    long nt = sysconf(_SC_NPROCESSORS_ONLN);
    const char *ev = getenv("OMP_NUM_THREADS");
    if (ev && atoi(ev) > 0) nt = atoi(ev);
    if (nt > 16) nt = 16;
    return nt < 1 ? 1u : (unsigned)nt;
}

typedef struct {
    void *arg;
    void (*fn)(void *, size_t, size_t);
    size_t i0, i1;
} host_job;

static void *host_job_run(void *p)
{
    host_job *j = (host_job *)p;
    j->fn(j->arg, j->i0, j->i1);
    return NULL;
}

/* fn(arg, i0, i1) over [0, n) in nt contiguous ranges */
static void host_parallel(unsigned nt, size_t n, void *arg, void (*fn)(void *, size_t, size_t))
{
    if (nt > n) nt = n ? (unsigned)n : 1u;
    host_job jobs[16];
    pthread_t th[16];
    int started[16] = {0};
    for (unsigned t = 0; t < nt; ++t) {
        jobs[t].arg = arg;
        jobs[t].fn = fn;
        jobs[t].i0 = n * t / nt;
        jobs[t].i1 = n * (t + 1) / nt;
    }
    for (unsigned t = 1; t < nt; ++t) started[t] = pthread_create(&th[t], NULL, host_job_run, &jobs[t]) == 0;
    host_job_run(&jobs[0]);
    for (unsigned t = 1; t < nt; ++t) {
        if (started[t]) pthread_join(th[t], NULL);
        else host_job_run(&jobs[t]);  /* no thread: run it here */
    }
}

typedef struct {
    const double *lik;
    uint32_t s;
    size_t se, sc;
    double *ex;
} exp_arg;

static void exp_range(void *p, size_t i0, size_t i1)
{
    exp_arg *a = (exp_arg *)p;
    for (size_t i = i0; i < i1; ++i) a->ex[i] = exp(a->lik[(i / a->s) * a->se + (i % a->s) * a->sc]);
}

/* main_MIDASPOM.c:413-425, on the s x s view lik[k*se + l*sc] (k = e row,
 * l = c column).  The exps of a large grid are evaluated in threads; the
 * weighted sum runs in the reference's order (k outer, l inner), so Ltot is
 * bit-identical to the sequential form in either layout. */
double mdp_log_total_view(const double *lik, uint32_t s, size_t se, size_t sc, double win)
{
    const size_t cells = (size_t)s * s;
    const unsigned nt = host_threads(cells);
    double *ex = nt > 1 ? (double *)malloc(sizeof(double) * cells) : NULL;
    if (ex) {
        exp_arg a = {lik, s, se, sc, ex};
        host_parallel(nt, cells, &a, exp_range);
    }
    double acc = 0;
    for (uint32_t k = 0; k < s; k++) {
        const double wk = (k == 0 || k == s - 1) ? 0.5 : 1.0;
        for (uint32_t l = 0; l < s; l++) {
            double w = wk;
            if (l == 0 || l == s - 1) w *= 0.5;
            acc += (ex ? ex[(size_t)k * s + l] : exp(lik[(size_t)k * se + (size_t)l * sc])) * w;
        }
    }
    free(ex);
    return 2 * log(win) + log(acc);
}

double mdp_log_total(const double *lik, uint32_t s, double win)
{
    return mdp_log_total_view(lik, s, s, 1, win);
}

typedef struct {
    const double *lik;
    uint32_t s;
    size_t se, sc;
    double ltot;
    int raw;
    uint32_t rows_per_part;
    size_t part0;   /* first part of the current batch */
    char **buf;     /* per part of the batch: the formatted text */
    size_t *len;
    size_t *cap;
    int fail;
} fmt_arg;

static void fmt_range(void *p, size_t q0, size_t q1)
{
    fmt_arg *a = (fmt_arg *)p;
    for (size_t q = q0; q < q1; ++q) {
        const size_t part = a->part0 + q;
        const uint32_t r0 = (uint32_t)(part * a->rows_per_part);
        uint32_t r1 = r0 + a->rows_per_part;
        if (r1 > a->s) r1 = a->s;
        size_t cap = a->cap[q], used = 0;
        char *b = a->buf[q];
        for (uint32_t i = r0; i < r1; i++) {
            for (uint32_t j = 0; j <= a->s; j++) {
                /* room for one cell: %.20lf of the largest double is 331 bytes */
                if (cap - used < 400) {
                    const size_t ncap = cap * 2 + 1024;
                    char *nb = (char *)realloc(b, ncap);
                    if (!nb) {
                        a->fail = 1;
                        a->buf[q] = b;
                        a->cap[q] = cap;
                        a->len[q] = 0;
                        return;
                    }
                    b = nb;
                    cap = ncap;
                }
                if (j == a->s) {
                    b[used++] = '\n';
                    break;
                }
                const double v = a->lik[(size_t)i * a->se + (size_t)j * a->sc];
                used += (size_t)snprintf(b + used, cap - used, "%.20lf\t", a->raw ? v : exp(v - a->ltot));
            }
        }
        a->buf[q] = b;
        a->cap[q] = cap;
        a->len[q] = used;
    }
}

/* main_MIDASPOM.c:427-436 (raw: the MPI build's Ltot == 0 branch,
 * main_MIDASPOM_MPI.c:527) on the view lik[i*se + j*sc] (i = e row, j = c
 * column).  Rows are cut into parts of about 256 KB of text; batches of a
 * few parts per thread are formatted in threads and written in order, so the
 * bytes are those of the sequential writer and the memory held at once is
 * bounded (a few MB per thread) whatever s is. */
int mdp_write_posterior_view(const char *path, const double *lik, uint32_t s, size_t se, size_t sc, double ltot,
                             int raw)
{
    FILE *f = fopen(path, "wb");
    if (!f) return mdp_set_error(MDP_EIO, "cannot open output file '%s'", path);
    const unsigned nt = host_threads((size_t)s * s);
    const size_t row_bytes = (size_t)s * 26u + 1u;
    uint32_t rpp = (uint32_t)((1u << 18) / row_bytes);
    if (rpp < 1) rpp = 1;
    if (rpp > s) rpp = s ? s : 1;
    const size_t nparts_all = s ? ((size_t)s + rpp - 1) / rpp : 0;
    const size_t batch = nt > 1 ? (size_t)nt * 4 : 1;  /* a few parts per thread */
    fmt_arg a = {lik, s, se, sc, ltot, raw, rpp, 0, (char **)calloc(batch, sizeof(char *)),
                 (size_t *)calloc(batch, sizeof(size_t)), (size_t *)calloc(batch, sizeof(size_t)), 0};
    int rc = MDP_OK;
    if (!a.buf || !a.len || !a.cap) rc = mdp_set_error(MDP_ENOMEM, "out of host memory");
    for (size_t p0 = 0; p0 < nparts_all && !rc; p0 += batch) {
        const size_t nb = nparts_all - p0 < batch ? nparts_all - p0 : batch;
        a.part0 = p0;
        host_parallel(nt, nb, &a, fmt_range);
        if (a.fail) rc = mdp_set_error(MDP_ENOMEM, "out of host memory");
        for (size_t q = 0; q < nb && !rc; ++q)
            if (a.len[q] && fwrite(a.buf[q], 1, a.len[q], f) != a.len[q]) rc = mdp_set_error(MDP_EIO, "write to '%s' failed", path);
    }
    if (a.buf)
        for (size_t q = 0; q < batch; ++q) free(a.buf[q]);
    free(a.buf);
    free(a.len);
    free(a.cap);
    if (fclose(f) != 0 && !rc) rc = mdp_set_error(MDP_EIO, "write to '%s' failed", path);
    return rc;
}

int mdp_write_posterior(const char *path, const double *lik, uint32_t s, double ltot, int raw)
{
    return mdp_write_posterior_view(path, lik, s, s, 1, ltot, raw);
}
