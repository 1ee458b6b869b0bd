/*
 * midaspom_amd/csrc/midaspom_cli.c -- `midaspom`, a drop-in for the
 * reference's bin_linux/MIDASPOM.out (and, with -g N, for
 * `mpirun -np N MIDASPOM_MPI.out`).
 *
 * Same getopt string, defaults and stdout lines as
 * /root/reference/sources/main_MIDASPOM.c:61-439; the posterior file has the
 * same bit layout (%.20lf\t per cell, \n per row).  The grid loop :341-395
 * runs on the GPU through the C ABI in include/midaspom.h.
 *
 * Extensions: -g <N> (or MIDASPOM_GPUS=N) splits the e rows into N
 * contiguous slabs (main_MIDASPOM_MPI.c:361-368) dealt round-robin over the
 * node's visible GPUs (N may exceed them: slabs then share a GPU, each on
 * its own stream).  MIDASPOM_TIMING=1 prints where the wall time went
 * (parse, HIP start-up, engine set-up incl. hipRTC, grid, Ltot, write) to
 * stderr.
 */
#include <ctype.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include <unistd.h>

#include "cli_exit.h"
#include "midaspom.h"

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int main(int argc, char **argv)
{
    const double t_start = now_s();
    const int timing = getenv("MIDASPOM_TIMING") && atoi(getenv("MIDASPOM_TIMING")) != 0;
    printf("------ MIDASPOM, beta version ------\n-> N. Alcala, E. M. Cole, and N. A. Rosenberg <-\n");

    float prior_occ = 0.5f;            /* -p, float32 as :66 */
    const char *fin = "input.txt";     /* -i */
    const char *fout = "posterior.txt";/* -o */
    double seg = 100;                  /* -d (code default, not the manual's 200) */
    unsigned nstep = 101;              /* -s */
    double mdisp = 400;                /* -m */
    double lo = 0.0, hi = 1.0;         /* -l, -u */
    int ngpu = 0;
    const char *env = getenv("MIDASPOM_GPUS");
    if (env) ngpu = atoi(env);

    int c;
    opterr = 0;
    while ((c = getopt(argc, argv, "m:p:d:i:o:s:l:u:g:")) != -1) {
        switch (c) {
        case 'm': mdisp = atof(optarg); break;
        case 'p': prior_occ = (float)atof(optarg); break;
        case 'd': seg = atof(optarg); break;
        case 'i': fin = optarg; break;
        case 'o': fout = optarg; break;
        case 's': nstep = (unsigned)atoi(optarg); break;
        case 'l': lo = atof(optarg); break;
        case 'u': hi = atof(optarg); break;
        case 'g': ngpu = atoi(optarg); break;
        case '?':
            /* message set of main_MIDASPOM.c:106-115 */
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
    if (nstep < 1) {  /* the reference indexes g[s - 1] (main_MIDASPOM.c:319): s = 0 is out of bounds there */
        fprintf(stderr, "midaspom: -s must be at least 1\n");
        return 1;
    }

    const double win = mdp_grid(nstep, lo, hi, NULL);
    printf("Parameters for numerical approximation of the posterior density:\n\tWindow size=%lf, number of steps=%d\n",
           win, nstep);

    printf("Reading observations from file %s... ", fin);
    mdp_model *model = NULL;
    int rc = mdp_model_load(fin, mdisp, prior_occ, seg, &model);
    if (rc) {
        fprintf(stderr, "\nmidaspom: %s\n", mdp_last_error());
        return 2;
    }
    mdp_problem pb;
    mdp_model_problem(model, &pb);
    printf("done\n");
    printf("Number of habitat patches: %d\nNumber of sampled years: %d\n", pb.n, pb.tmax);

    printf("Dispersal matrix:\n");
    for (unsigned i = 0; i < pb.n; i++) {
        for (unsigned j = 0; j < pb.n; j++) printf("%.3f ", pb.M[(size_t)i * pb.n + j]);
        printf("\n");
    }
    printf("Input occupancy data:\n");
    for (unsigned t = 0; t < pb.tmax; t++) {
        printf("Year %d: ", t);
        for (unsigned j = 0; j < pb.n; j++) printf("%d ", pb.obs[(size_t)t * pb.n + j]);
        printf("\n");
    }
    printf("Number of possible states per year:\n");
    for (unsigned t = 0; t < pb.tmax; t++) printf("Year %d: %d\n", t, pb.year_off[t + 1] - pb.year_off[t]);
    printf("Number of states to compute: %d\n", 1u << pb.nvar);

    double *grid = (double *)malloc(sizeof(double) * nstep);
    double *lik = (double *)malloc(sizeof(double) * (size_t)nstep * nstep);
    if (!grid || !lik) {
        fprintf(stderr, "midaspom: out of host memory\n");
        return 2;
    }
    mdp_grid(nstep, lo, hi, grid);
    setbuf(stdout, NULL);

    time_t start, end;
    time(&start);
    printf("Starting parallel likelihood computation\n");
    const double t_parsed = now_s();
    mdp_engine *eng = NULL;
    int *devs = NULL;
    if (ngpu > 0) {  /* slabs round-robin over the visible GPUs */
        const int nvis = mdp_device_count();
        devs = (int *)malloc(sizeof(int) * (size_t)ngpu);
        if (!devs) {
            fprintf(stderr, "midaspom: out of host memory\n");
            return 2;
        }
        for (int i = 0; i < ngpu; i++) devs[i] = nvis > 0 ? i % nvis : i;
    } else {
        (void)mdp_device_count();  /* HIP start-up, timed on its own */
    }
    const double t_hip = now_s();
    rc = mdp_engine_create(&pb, devs, ngpu > 0 ? ngpu : 0, &eng);
    const double t_setup = now_s();
    /* lik[c][e]: each GPU writes its slab's columns contiguously (the
     * layout the kernels store fastest); Ltot and the writer read it in
     * place through the transposed view, so the file is the same bytes */
    if (!rc) rc = mdp_loglik_grid_layout(eng, grid, nstep, grid, nstep, MDP_LAYOUT_CE, lik);
    free(devs);
    if (rc) {
        fprintf(stderr, "midaspom: %s\n", mdp_last_error());
        mdp_engine_destroy(eng);
        return 3;
    }
    const double t_run = now_s();
    mdp_engine_destroy(eng);
    const double t_grid = now_s();
    for (unsigned ie = 0; ie < nstep; ie++) printf("%.2f%% done\n", ((float)ie + 1) * 100.0 / nstep);
    printf("end likelihood computation\n");

    const double ltot = mdp_log_total_view(lik, nstep, 1, nstep, win);
    const double t_ltot = now_s();
    printf("Total log-likelihood=%.5lf\n", ltot);
    printf("Writing output in file %s... ", fout);
    rc = mdp_write_posterior_view(fout, lik, nstep, 1, nstep, ltot, 0);
    if (rc) {
        fprintf(stderr, "midaspom: %s\n", mdp_last_error());
        return 2;
    }
    if (timing)
        fprintf(stderr,
                "midaspom timing (s): parse %.3f hip_init %.3f setup %.3f grid %.3f destroy %.3f ltot %.3f write %.3f "
                "total %.3f\n",
                t_parsed - t_start, t_hip - t_parsed, t_setup - t_hip, t_run - t_setup, t_grid - t_run, t_ltot - t_grid,
                now_s() - t_ltot, now_s() - t_start);
    time(&end);
    printf("done\n Total running time: %.2lf min\n", difftime(end, start) / 60.0);
    free(grid);
    free(lik);
    mdp_model_free(model);
    /* absolute CLOCK_MONOTONIC stamps of main's entry and return: a parent
     * timing the process on the same clock attributes the wall outside main
     * (exec, loader, library constructors; exit handlers, runtime teardown) */
    if (timing) fprintf(stderr, "midaspom clock (s): main_entry %.6f main_return %.6f\n", t_start, now_s());
    /* the posterior file is closed: leave without the HIP runtime's
     * exit-time teardown unless a tool needs the exit handlers (cli_exit.h) */
    mdp_cli_leave(0);
    return 0;
}
