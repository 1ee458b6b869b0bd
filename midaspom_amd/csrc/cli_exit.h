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
 */
#ifndef MIDASPOM_CLI_EXIT_H
#define MIDASPOM_CLI_EXIT_H

#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

static inline int mdp_cli_env_set(const char *name)
{
    const char *v = getenv(name);
    return v && *v;
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
    _exit(code);
}

#endif
