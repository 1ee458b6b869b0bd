/*
 * midaspom_amd/csrc/midaspom_future_cli.c -- drop-in for the reference's
 * bin_linux/MIDASPOM_future.out (/root/reference/sources/main_MIDASPOM_future.c:113-415):
 * same getopt string ("n:a:m:p:q:d:i:o:S:s:D:", :140) and code defaults
 * (:123-133; the code's -D 1, not the manual's 0), same stdout lines and
 * output layout ("%d\t" per future year, no newline, :402-404).  The
 * replicate loop runs on the GPU through mdp_future_simulate.
 *
 * Extensions (the reference has no other way to set them):
 *   -g <N>     GPUs (or MIDASPOM_GPUS=N): the replicates in N contiguous
 *              ranges (remainder to the first, the MIDASPOM_future_MPI.out
 *              partition, future_MPI.c:376-383), one host thread and engine
 *              per range, the ranges dealt round-robin over the visible GPUs;
 *              replicate r draws from the stream addressed by (seed, r), so
 *              the counts do not depend on N
 *   -r <seed>  generator seed; default time(NULL) like srand(time(NULL))
 *              (:345), or $MIDASPOM_SEED.  The draws are Philox streams, not
 *              glibc rand(): runs are reproducible per seed and agree with
 *              the reference statistically.
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

struct range {
    const int32_t *pend;
    const double *post;
    uint32_t n, necstep, tfut;
    double mdisp, d, KD, KS, dS;
    int dev;
    unsigned long long seed;
    uint64_t rep0, nrep;
    uint64_t *cnt;  /* [tfut] */
    int rc;
    char err[256];
};

static void *run_range(void *arg)
{
    struct range *r = arg;
    mdp_future *f = NULL;
    r->rc = mdp_future_create(r->pend, r->n, r->post, r->necstep, r->mdisp, r->d, r->KD, r->KS, r->dS, r->dev, &f);
    if (r->rc == MDP_OK && r->nrep) r->rc = mdp_future_simulate(f, r->seed, r->rep0, r->nrep, r->tfut, r->cnt);
    if (r->rc != MDP_OK) snprintf(r->err, sizeof r->err, "%s", mdp_last_error());
    mdp_future_destroy(f);
    return NULL;
}

int main(int argc, char **argv)
{
    printf("------MIDASPOM, beta MPI version -------\n-> N. Alcala, E. M. Cole, N. A. Rosenberg  <-\n");
    time_t start, end;
    int tfut = 50, nsimul = 10000, ngpu = 1;
    if (getenv("MIDASPOM_GPUS")) ngpu = atoi(getenv("MIDASPOM_GPUS"));
    double KS = 0, dS = 200, KD = 1, mdisp = 400.0, d = 200;
    float prioroc = 0.5f;
    const char *finame = "posterior.txt", *fname = "input.txt", *fout = "pext_future.txt";
    const char *env_seed = getenv("MIDASPOM_SEED");
    unsigned long long seed = env_seed ? strtoull(env_seed, NULL, 0) : (unsigned long long)time(NULL);
    int c;
    opterr = 0;
    while ((c = getopt(argc, argv, "n:a:m:p:q:d:i:o:S:s:D:g:r:")) != -1) {
        switch (c) {
        case 'n': nsimul = atoi(optarg); break;
        case 'a': tfut = atoi(optarg); break;
        case 'm': mdisp = atof(optarg); break;
        case 'p': prioroc = (float)atof(optarg); break;
        case 'q': finame = optarg; break;
        case 'd': d = atof(optarg); break;
        case 'i': fname = optarg; break;
        case 'o': fout = optarg; break;
        case 'S': KS = atof(optarg); break;
        case 's': dS = atof(optarg); break;
        case 'D': KD = atof(optarg); break;
        case 'g': ngpu = atoi(optarg); break;
        case 'r': seed = strtoull(optarg, NULL, 0); break;
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
    printf("%d years in the future\n", tfut);
    printf("Reading observations from file %s... ", fname);
    uint32_t n, tmax, necstep;
    int32_t *pend;
    double *post;
    if (mdp_future_read_survey(fname, &n, &tmax, &pend) != MDP_OK) {
        fprintf(stderr, "%s\n", mdp_last_error());
        return 1;
    }
    printf("Last occupancy survey:\n");
    for (uint32_t j = 0; j < n; ++j) printf("%d ", pend[j]);
    printf("\n");
    printf("\n done\n");
    printf("Number of habitat patches: %u\nNumber of sampled years: %u\n", n, tmax);
    printf("Reading posterior distribution from file %s... ", finame);
    if (mdp_future_read_posterior(finame, &necstep, &post) != MDP_OK) {
        fprintf(stderr, "%s\n", mdp_last_error());
        return 1;
    }
    printf("%uX%u posterior distribution\n", necstep, necstep);
    /* migration matrix with the source row (:265-284) */
    const double a = 1.0 / mdisp;
    printf("Migration matrix:\n");
    for (uint32_t i = 0; i < n + 1; ++i) {
        for (uint32_t j = 0; j < n; ++j) {
            double v;
            if (i == n) v = exp(-a * (j + 1) * dS);
            else if (i == j) v = 0.0;
            else v = exp(-a * (i < j ? j - i : i - j) * d);
            printf("%.3f ", v);
        }
        printf("\n");
    }
    /* completions of the last survey and their (unused) priors (:286-332) */
    unsigned nm = 0;
    for (uint32_t j = 0; j < n; ++j) nm += pend[j] == -1;
    const unsigned np = nm < 31 ? 1u << nm : 0;
    printf("npstates = %u\n", np);
    printf("Last occupancy survey:\n");
    for (unsigned k = 0; k < np; ++k) {
        printf("\t");
        double pr = 1;
        unsigned q = 0;
        for (uint32_t j = 0; j < n; ++j) {
            int v = pend[j];
            if (pend[j] == -1) {
                const unsigned bit = (k >> (nm - 1 - q)) & 1u;
                ++q;
                v = (int)bit;
                pr *= (float)bit * prioroc + (float)(1 - bit) * (1 - prioroc);
            }
            printf("%d ", v);
        }
        printf("; pr=%lf\n", pr);
    }
    int *lik = calloc(tfut > 0 ? (size_t)tfut : 1, sizeof(int));
    time(&start);
    printf("Starting likelihood computation\n");
    int rc = MDP_OK;
    if (tfut > 0 && nsimul > 0) {
        if (ngpu < 1) ngpu = 1;
        if (ngpu > nsimul) ngpu = nsimul;
        const int ndev = mdp_device_count() > 0 ? mdp_device_count() : 1;
        struct range *rg = calloc((size_t)ngpu, sizeof *rg);
        pthread_t *th = calloc((size_t)ngpu, sizeof *th);
        char *started = calloc((size_t)ngpu, 1);
        const uint64_t avg = (uint64_t)nsimul / (uint64_t)ngpu, rem = (uint64_t)nsimul % (uint64_t)ngpu;
        for (int r = 0; r < ngpu; ++r) {
            const uint64_t r0 = r == 0 ? 0 : (uint64_t)r * avg + rem, r1 = (uint64_t)(r + 1) * avg + rem;
            rg[r] = (struct range){pend, post, n, necstep, (uint32_t)tfut, mdisp, d, KD, KS, dS, r % ndev, seed,
                                   r0, r1 - r0, calloc((size_t)tfut, sizeof(uint64_t)), 0, ""};
        }
        for (int r = 1; r < ngpu; ++r) started[r] = pthread_create(&th[r], NULL, run_range, &rg[r]) == 0;
        run_range(&rg[0]);
        for (int r = 1; r < ngpu; ++r) {
            if (started[r]) pthread_join(th[r], NULL);
            else run_range(&rg[r]);  // no thread: this range runs here, after the others
        }
        for (int r = 0; r < ngpu; ++r) {
            if (rg[r].rc != MDP_OK && rc == MDP_OK) {
                rc = rg[r].rc;
                fprintf(stderr, "GPU future simulation failed: %s\n", rg[r].err);
            }
            for (int t = 0; t < tfut; ++t) lik[t] += (int)rg[r].cnt[t];
            free(rg[r].cnt);
        }
        free(rg), free(th), free(started);
    }
    if (rc != MDP_OK) return 1;
    printf("end likelihood computation\n");
    printf("Writing on file %s... ", fout);
    FILE *fe = fopen(fout, "wb");
    if (!fe) {
        fprintf(stderr, "cannot write %s\n", fout);
        return 1;
    }
    for (int t = 0; t < tfut; ++t) fprintf(fe, "%d\t", lik[t]);
    fclose(fe);
    printf("done\n");
    time(&end);
    printf("Finished. It took  %.2lf min\n", difftime(end, start) / 60.0);
    free(lik);
    mdp_free(pend);
    mdp_free(post);
    /* without the HIP runtime's exit-time teardown unless a tool needs the
     * exit handlers (cli_exit.h) */
    mdp_cli_leave(0);
    return 0;
}
