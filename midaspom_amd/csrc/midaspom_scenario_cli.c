/*
 * midaspom_amd/csrc/midaspom_scenario_cli.c -- drop-ins for the reference's
 * scenario programs, built twice:
 *   SCN_KIND 0: `midaspom_dieoff` for bin_linux/MIDASPOM_dieoff.out
 *               (/root/reference/sources/main_MIDASPOM_dieoff.c:94-384)
 *   SCN_KIND 1: `midaspom_loss`   for bin_linux/MIDASPOM_loss.out
 *               (/root/reference/sources/main_MIDASPOM_loss.c:115-421)
 * Same getopt strings, code defaults, stdout lines and output layout
 * ("%.20lf\t" per value; loss: one row per K, "\n" per row).  The likelihood
 * runs on the GPU through mdp_scenario_lik (include/midaspom.h).
 *
 * Policy: the reference leaves tdis, eB and cB uninitialised
 * when -a, -e or -c is omitted; here they are required.
 *
 * Extension: -g <N> (or MIDASPOM_GPUS=N) splits the K grid into N contiguous
 * slabs (remainder to the first, the MIDASPOM_{dieoff,loss}_MPI.out
 * partition, dieoff_MPI.c:323-330), one host thread and engine per slab, the
 * slabs dealt round-robin over the visible GPUs; the output is the same file.
 */
#include <ctype.h>
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include <unistd.h>

#include "cli_exit.h"
#include "midaspom.h"

#ifndef SCN_KIND
#define SCN_KIND 0
#endif

struct slab {
    const int32_t *row;
    unsigned n, nK, nd;
    double mdisp, d, eB, cB;
    float prioroc;
    int ts, tdis, dev;
    const double *K, *dv;
    double *L;
    int rc;
    char err[256];
};

static void *run_slab(void *arg)
{
    struct slab *sl = arg;
    mdp_scenario *sc = NULL;
    sl->rc = mdp_scenario_create(sl->row, sl->n, sl->mdisp, sl->prioroc, sl->d, SCN_KIND, sl->dev, &sc);
    if (sl->rc == MDP_OK && sl->nK)
        sl->rc = mdp_scenario_lik(sc, sl->ts, sl->tdis, &sl->eB, 1, &sl->cB, 1, sl->K, sl->nK, sl->dv, sl->nd, sl->L);
    if (sl->rc != MDP_OK) snprintf(sl->err, sizeof sl->err, "%s", mdp_last_error());
    mdp_scenario_destroy(sc);
    return NULL;
}

int main(int argc, char **argv)
{
#if SCN_KIND == 0
    printf("------ MIDASPOM, in situ die-off hypothesis, beta version -------\n-> N. Alcala, E. M. Cole, N. A. "
           "Rosenberg <-\n");
    const char *opts = "b:a:e:c:m:p:d:i:o:s:l:u:g:";
    const char *fout = "lh_dieoff.txt";
#else
    printf("------ MIDASPOM, habitat loss hypothesis, beta version -------\n-> N. Alcala, E. M. Cole, N. A. "
           "Rosenberg  <-\n");
    const char *opts = "b:a:e:c:m:p:d:i:o:s:v:l:u:L:U:g:";
    const char *fout = "lh_loss.txt";
#endif
    int ts = 20, tdis = 0, have_a = 0, have_e = 0, have_c = 0, ngpu = 1;
    if (getenv("MIDASPOM_GPUS")) ngpu = atoi(getenv("MIDASPOM_GPUS"));
    unsigned nstep = 151, nstepd = 20;
    double eB = 0, cB = 0, Kmin = 0.1, Kmax = 100.0, mdisp = 400.0, d = 200, dmin = 200, dmax = 4000;
    float prioroc = 0.5f;
    const char *fname = "input.txt";
    int c;
    opterr = 0;
    while ((c = getopt(argc, argv, opts)) != -1) {
        switch (c) {
        case 'b': ts = atoi(optarg); break;
        case 'a': tdis = atoi(optarg), have_a = 1; break;
        case 'e': eB = atof(optarg), have_e = 1; break;
        case 'c': cB = atof(optarg), have_c = 1; break;
        case 'm': mdisp = atof(optarg); break;
        case 'p': prioroc = (float)atof(optarg); break;
        case 'd': d = atof(optarg); break;
        case 'i': fname = optarg; break;
        case 'o': fout = optarg; break;
        case 's': nstep = (unsigned)atoi(optarg); break;
        case 'v': nstepd = (unsigned)atoi(optarg); break;
        case 'l': Kmin = atof(optarg); break;
        case 'u': Kmax = atof(optarg); break;
        case 'L': dmin = atof(optarg); break;
        case 'U': dmax = atof(optarg); break;
        case 'g': ngpu = atoi(optarg); break;
        case '?':
            if (optopt == 'c')
                fprintf(stderr, "Option -%c requires an argument.\n", optopt);
            else if (isprint(optopt))
                fprintf(stderr, "Unknown option `-%c'.\n", optopt);
            else
                fprintf(stderr, "Unknown option character `\\x%x'.\n", optopt);
            return 1;
        default:
            abort();
        }
    }
    if (!have_a || !have_e || !have_c) {
        fprintf(stderr, "Options -a (years after the event), -e and -c are required.\n");
        return 1;
    }
#if SCN_KIND == 0
    printf("%d years before increased die-off, %d years after increased die-off\n", ts, tdis);
#else
    printf("%d years before habitat loss, %d years after the loss\n", ts, tdis);
#endif
    printf("Reading observations from file %s... ", fname);
    FILE *fo = fopen(fname, "rb");
    if (!fo) {
        fprintf(stderr, "cannot open %s\n", fname);
        return 1;
    }
    unsigned n = 1;
    while ((c = fgetc(fo)) != EOF) {  /* dieoff.c:186-191 */
        if (c == '\n') break;
        if (c == ' ' || c == '\t') n++;
    }
    fclose(fo);
#if SCN_KIND == 1
    printf("%u patches\n", n);
    printf("Reading observations from file %s... ", fname);
#endif
    int32_t *row = malloc(n * sizeof(int32_t));
    fo = fopen(fname, "rb");
    for (unsigned j = 0; j < n; ++j) /* first survey row only, dieoff.c:196-198 */
        if (fscanf(fo, "%d", &row[j]) != 1) row[j] = 0;
    fclose(fo);
    printf("done\n");
    /* observed states and priors for the log lines (dieoff.c:205-232) */
    unsigned nm = 0;
    for (unsigned j = 0; j < n; ++j) nm += row[j] == -1;
    const unsigned np = 1u << nm;
    unsigned *ps = calloc(np, sizeof(unsigned));
    float *pr = malloc(np * sizeof(float));
    for (unsigned k = 0; k < np; ++k) pr[k] = 1;
    unsigned s1 = 0;
    for (unsigned j = 0; j < n; ++j) {
        if (row[j] == -1) s1++;
        for (unsigned k = 0; k < np; ++k) {
            if (row[j] > -1) {
                ps[k] += (unsigned)row[j] << (n - j - 1);
            } else {
                const unsigned st1 = np >> s1, b = k / st1 % 2;
                ps[k] += b << (n - j - 1);
                pr[k] *= b * prioroc + (1 - b) * (1 - prioroc);
            }
        }
    }
#if SCN_KIND == 0
    printf("%u patches\n", n);
#endif
    printf("Migration matrix:\n");
    const double a = 1.0 / mdisp;
    for (unsigned i = 0; i < n; ++i) {
        for (unsigned j = 0; j < n; ++j) printf("%.3f ", i == j ? 0.0 : exp(-a * (double)(i > j ? i - j : j - i) * d));
        printf("\n");
    }
#if SCN_KIND == 1
    printf("First occupancy survey:\n");
#endif
    for (unsigned k = 0; k < np; ++k) {
#if SCN_KIND == 1
        printf("\t");
#endif
        for (unsigned j = 0; j < n; ++j) printf("%u ", (ps[k] >> (n - 1 - j)) & 1u);
        printf("; pr=%lf\n", pr[k]);
    }
    double *K = malloc(nstep * sizeof(double)), *dv = malloc(nstepd * sizeof(double));
    mdp_kgrid(nstep, Kmin, Kmax, K);
    mdp_dgrid(nstepd, dmin, dmax, dv);
    time_t start, end;
    time(&start);
    printf("Starting likelihood computation\n");
    const unsigned nd = SCN_KIND == 1 ? nstepd : 1u;
    double *L = malloc((size_t)nstep * nd * sizeof(double));
    if (ngpu < 1) ngpu = 1;
    if ((unsigned)ngpu > nstep) ngpu = (int)(nstep ? nstep : 1);
    struct slab *sl = calloc((size_t)ngpu, sizeof *sl);
    pthread_t *th = calloc((size_t)ngpu, sizeof *th);
    const unsigned avg = nstep / (unsigned)ngpu, rem = nstep % (unsigned)ngpu;
    for (int r = 0; r < ngpu; ++r) {
        const unsigned k0 = r == 0 ? 0 : (unsigned)r * avg + rem, k1 = (unsigned)(r + 1) * avg + rem;
        sl[r] = (struct slab){row, n, k1 - k0, nd, mdisp, d, eB, cB, prioroc, ts, tdis, r, K + k0, dv,
                              L + (size_t)k0 * nd, 0, ""};
    }
    {   /* slabs dealt round-robin over the visible devices */
        const int ndev = mdp_device_count() > 0 ? mdp_device_count() : 1;
        for (int r = 0; r < ngpu; ++r) sl[r].dev = r % ndev;
    }
    char *started = calloc((size_t)ngpu, 1);
    for (int r = 1; r < ngpu; ++r) started[r] = pthread_create(&th[r], NULL, run_slab, &sl[r]) == 0;
    run_slab(&sl[0]);
    for (int r = 1; r < ngpu; ++r) {
        if (started[r]) pthread_join(th[r], NULL);
        else run_slab(&sl[r]);  // no thread: this slab runs here, after the others
    }
    free(started);
    for (int r = 0; r < ngpu; ++r)
        if (sl[r].rc != MDP_OK) {
            fprintf(stderr, "midaspom: %s\n", sl[r].err);
            return 1;
        }
    free(sl);
    free(th);
    printf("end likelihood computation\n");
    printf("Writing on file %s... ", fout);
    FILE *fe = fopen(fout, "wb");
    if (!fe) {
        fprintf(stderr, "cannot write %s\n", fout);
        return 1;
    }
    for (unsigned i = 0; i < nstep; ++i) {
        for (unsigned j = 0; j < nd; ++j) fprintf(fe, "%.20lf\t", L[(size_t)i * nd + j]);
#if SCN_KIND == 1
        fprintf(fe, "\n");
#endif
    }
    fclose(fe);
    printf("done\n");
    time(&end);
    printf("Finished. It took  %.2lf min\n", difftime(end, start) / 60.0);
    free(row), free(ps), free(pr), free(K), free(dv), free(L);
    /* without the HIP runtime's exit-time teardown unless a tool needs the
     * exit handlers (cli_exit.h) */
    mdp_cli_leave(0);
    return 0;
}
