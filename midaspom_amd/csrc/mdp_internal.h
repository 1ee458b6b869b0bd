/* midaspom_amd/csrc/mdp_internal.h -- internals shared by the host C code and
 * the HIP engine (not part of the public ABI). */
#ifndef MDP_INTERNAL_H
#define MDP_INTERNAL_H
#include "midaspom.h"

#ifdef __cplusplus
extern "C" {
#endif

/* printf-style setter for the thread-local error string; returns code. */
int mdp_set_error(int code, const char *fmt, ...);

struct mdp_model {
    uint32_t n, tmax, nvar, nextid;
    int32_t *obs;          /* [tmax][n]                    */
    uint32_t *var_cols;    /* [nvar]                       */
    double *M;             /* [n][n]                       */
    uint32_t *short_state; /* [nextid]                     */
    uint32_t *year_off;    /* [tmax+1]                     */
    uint32_t *year_ids;    /* [year_off[tmax]]             */
    float *prior;          /* [year_off[1]]                */
};

#ifdef __cplusplus
}
#endif
#endif
