/* oracle/spom_oracle.h -- TEST INFRASTRUCTURE ONLY: CPU restatement of the
 * reference MIDASPOM likelihood (see spom_oracle.c header). */
#ifndef SPOM_ORACLE_H
#define SPOM_ORACLE_H
#include <stddef.h>

#define ORC_EIO -1
#define ORC_ENOMEM -2
#define ORC_EINVAL -3

typedef struct orc_model {
    unsigned n, tmax, nvar, nstates, nextid;
    int *obs;               /* [tmax][n] parsed observations            */
    unsigned *isvar;        /* [n] column ever non-zero                  */
    double *M;              /* [n][n] dispersal kernel                   */
    unsigned *colw;         /* [n] bit weight of a column in a state id  */
    unsigned *np;           /* [tmax] observed states per year           */
    unsigned *yoff;         /* [tmax+1] offsets into simp                */
    float *prior;           /* [np[0]] float32 prior of year-0 states    */
    unsigned *simp;         /* [sum np] short ids per year               */
    unsigned *short2all;    /* [nextid] full state id of each short id   */
    unsigned char *piall;   /* [nstates][n] state bits                   */
} orc_model;

int orc_parse(const char *path, unsigned *n, unsigned *tmax, int **obs);
int orc_model_build(const int *obs, unsigned n, unsigned tmax, double m, float p, double d,
                    orc_model **out);
int orc_model_load(const char *path, double m, float p, double d, orc_model **out);
void orc_model_free(orc_model *md);
double orc_grid(unsigned s, double lo, double hi, double *g);
int orc_loglik_rows(const orc_model *md, const double *eg, const double *cg, unsigned s,
                    unsigned ie0, unsigned ie1, double *out);
int orc_loglik_points(const orc_model *md, const double *e, const double *c, size_t npts,
                      double *out);
int orc_loglik_grid_mt(const orc_model *md, const double *eg, const double *cg, unsigned s,
                       unsigned nthreads, double *out);
double orc_ltot(const double *lik, unsigned s, double win);
int orc_write_posterior(const char *path, const double *lik, unsigned s, double ltot);
int orc_run(const char *in_path, const char *out_path, double m, double p, double d,
            unsigned s, double lo, double hi, unsigned nthreads, double *lik_out,
            double *ltot_out);
#endif
