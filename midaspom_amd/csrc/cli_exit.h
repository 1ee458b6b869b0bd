/*
 * midaspom_amd/csrc/cli_exit.h -- how the drop-in CLIs leave main.
 *
 * By default they flush and _exit(0): the HIP runtime's exit-time teardown
 * (its static destructors release every queue and allocation one by one)
 * took 40-120 ms after main returned, more than the whole grid on config 1,
 * and the kernel driver frees the process's device state on exit either way.
 * _exit also skips every other atexit handler, so the CLIs return from main
 * normally instead when
 *   - MIDASPOM_FULL_EXIT=1 is set, or
 *   - a tool that writes its results at exit is attached: rocprofv3 /
 *     rocprofiler-sdk (ROCP_TOOL_LIBRARIES, set by rocprofv3) or gcov
 *     (GCOV_PREFIX / GCOV_PREFIX_STRIP).
 *
 * Before the _exit the host's cores are woken (round 6): on the GPU pool's
 * boxes a process that holds a HIP context takes 40-70 ms to be reaped after
 * _exit -- the same for a bare device-count program, with or without a
 * context touch, after 0-400 ms of sleep -- unless several host cores were
 * busy just before it exits: 16 threads spinning 2 ms and joined cut it to
 * 1 ms, 2 threads or one idle thread do not; in the CLI on config 1 (s = 50)
 * 16 x 0.5 ms, 8 x 2 ms and 4 x 2 ms all take the remainder from 74 ms to
 * 2-4 ms, counting the spin (scripts/exit_probe.py,
 * profiles/r06/analysis/exit_probe_*.jsonl).  The CLI's own writer and
 * normaliser run threads on grids of 256^2 cells and more, which is why its
 * exit was fast there and slow below (round 5's open question: s = 255 pays
 * 69 ms, s = 256 1 ms).  The cause is in the kernel's exit path, not in this
 * code.  MIDASPOM_EXIT_WARM=<threads>[,<microseconds>] changes the default
 * 16 x 500 us (0: off).
 */
#ifndef MIDASPOM_CLI_EXIT_H
#define MIDASPOM_CLI_EXIT_H

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include <unistd.h>

static inline int mdp_cli_env_set(const char *name)
{
    const char *v = getenv(name);
    return v && *v;
}

static inline double mdp_cli_now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void *mdp_cli_spin(void *p)
{
    const double until = mdp_cli_now() + *(const double *)p;
    volatile unsigned long n = 0;
    while (mdp_cli_now() < until) ++n;
    return NULL;
}

/* wake `threads` host cores for `us` microseconds each (joined) */
static inline void mdp_cli_warm_cores(void)
{
    int threads = 16, us = 500;
    const char *w = getenv("MIDASPOM_EXIT_WARM");
    if (w && *w) {
        threads = atoi(w);
        const char *c = w;
        while (*c && *c != ',') ++c;
        if (*c == ',') us = atoi(c + 1);
    }
    if (threads <= 0 || us <= 0) return;
    if (threads > 64) threads = 64;
    const double secs = 1e-6 * (double)us;
    pthread_t th[64];
    int ok[64] = {0};
    for (int i = 0; i < threads; i++) ok[i] = pthread_create(&th[i], NULL, mdp_cli_spin, (void *)&secs) == 0;
    for (int i = 0; i < threads; i++)
        if (ok[i]) pthread_join(th[i], NULL);
}

/* leave now with `code` (fast path), or return so main can return it */
static inline void mdp_cli_leave(int code)
{
    const char *full = getenv("MIDASPOM_FULL_EXIT");
    if ((full && atoi(full) != 0) || mdp_cli_env_set("ROCP_TOOL_LIBRARIES") || mdp_cli_env_set("GCOV_PREFIX") ||
        mdp_cli_env_set("GCOV_PREFIX_STRIP"))
        return;
    fflush(stdout);
    fflush(stderr);
    mdp_cli_warm_cores();
    _exit(code);
}

#endif
