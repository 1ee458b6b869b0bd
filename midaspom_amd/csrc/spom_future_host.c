/*
 * midaspom_amd/csrc/spom_future_host.c -- input readers of the future
 * program (host side; the simulation runs on the GPU, spom_future.hip).
 *
 * Reference regions (/root/reference/sources/main_MIDASPOM_future.c):
 *   mdp_future_read_survey     :193-225  n from the separators of line 1,
 *                                        tmax from '\n', then tmax*n "%d"
 *                                        tokens streamed across lines (Q6);
 *                                        the LAST n tokens are the survey
 *   mdp_future_read_posterior  :237-262  necstep = separators on line 1 (the
 *                                        writer's trailing tab makes it s),
 *                                        then necstep^2 "%lf" values
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mdp_internal.h"

static char *slurp(const char *path, size_t *len)
{
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    size_t cap = 1 << 16, got = 0;
    char *buf = (char *)malloc(cap + 1);
    while (buf) {
        size_t r = fread(buf + got, 1, cap - got, f);
        got += r;
        if (got < cap) break;
        cap *= 2;
        char *nb = (char *)realloc(buf, cap + 1);
        if (!nb) { free(buf); buf = NULL; break; }
        buf = nb;
    }
    fclose(f);
    if (buf) buf[got] = 0;
    *len = got;
    return buf;
}

int mdp_future_read_survey(const char *path, uint32_t *n_out, uint32_t *tmax_out, int32_t **row_out)
{
    if (!path || !n_out || !tmax_out || !row_out) return mdp_set_error(MDP_EINVAL, "null argument");
    size_t len;
    char *buf = slurp(path, &len);
    if (!buf) return mdp_set_error(MDP_EIO, "cannot open input file '%s'", path);
    uint32_t n = 1, tmax = 0;
    for (size_t q = 0; q < len; q++) {
        if (buf[q] == '\n') tmax++;
        else if (tmax == 0 && (buf[q] == ' ' || buf[q] == '\t')) n++;
    }
    int32_t *row = (int32_t *)calloc(n, sizeof(int32_t));
    if (!row) { free(buf); return mdp_set_error(MDP_ENOMEM, "out of host memory"); }
    /* :217-224: pend[j] is overwritten row after row; a token that does not
     * parse ends the stream and the cells keep their last values */
    const char *p = buf;
    for (size_t q = 0; q < (size_t)tmax * n; q++) {
        char *end;
        while (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r' || *p == '\v' || *p == '\f') p++;
        if (!*p) break;
        long v = strtol(p, &end, 10);
        if (end == p) break;
        row[q % n] = (int32_t)v;
        p = end;
    }
    free(buf);
    *n_out = n, *tmax_out = tmax, *row_out = row;
    return MDP_OK;
}

int mdp_future_read_posterior(const char *path, uint32_t *necstep_out, double **post_out)
{
    if (!path || !necstep_out || !post_out) return mdp_set_error(MDP_EINVAL, "null argument");
    size_t len;
    char *buf = slurp(path, &len);
    if (!buf) return mdp_set_error(MDP_EIO, "cannot open posterior file '%s'", path);
    uint32_t s = 0;
    for (size_t q = 0; q < len && buf[q] != '\n'; q++)
        if (buf[q] == ' ' || buf[q] == '\t') s++;
    double *post = (double *)malloc(((size_t)s * s + 1) * sizeof(double));
    if (!post) { free(buf); return mdp_set_error(MDP_ENOMEM, "out of host memory"); }
    const char *p = buf;
    size_t got = 0;
    for (; got < (size_t)s * s; got++) {
        char *end;
        double v = strtod(p, &end); /* "%lf": skips whitespace, reads -nan / inf too */
        if (end == p) break;
        post[got] = v;
        p = end;
    }
    free(buf);
    if (got < (size_t)s * s) {
        free(post);
        return mdp_set_error(MDP_EINVAL, "posterior '%s': %zu of %u x %u values", path, got, s, s);
    }
    *necstep_out = s, *post_out = post;
    return MDP_OK;
}

void mdp_free(void *p) { free(p); }
