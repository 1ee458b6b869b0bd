/* Floor of a HIP command-line program: load the runtime, count the devices
 * (HIP start-up), optionally touch device 0 (context), optionally sleep
 * (sleep=<ms>: is the exit's cost a background task started with the
 * runtime, which a longer-lived process hides?), then exit normally or by
 * _exit (no runtime teardown).  Prints main's entry / return on
 * CLOCK_MONOTONIC so the parent can time the exit.
 * thread: create and join one host thread before the exit (the drop-in CLI's
 * writer uses threads on grids of 256^2 cells and more, where its exit is fast).
 * pool=N: N threads busy 2 ms each, joined.
 * Usage: hipinit_probe [ctx] [fast] [sleep=<ms>] [thread] [pool=N] */
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void *noop(void *p) { return p; }
static void *spin(void *p)
{
    const double t0 = now_s();
    volatile double x = 0;
    while (now_s() - t0 < 0.002) x += 1.0;
    return p;
}

int main(int argc, char **argv)
{
    int ctx = 0, fast = 0, sleep_ms = 0, thread = 0, pool = 0;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "ctx")) ctx = 1;
        if (!strcmp(argv[i], "fast")) fast = 1;
        if (!strncmp(argv[i], "sleep=", 6)) sleep_ms = atoi(argv[i] + 6);
        if (!strcmp(argv[i], "thread")) thread = 1;
        if (!strncmp(argv[i], "pool=", 5)) pool = atoi(argv[i] + 5);
    }
    const double t0 = now_s();
    int n = 0;
    hipGetDeviceCount(&n);
    const double t1 = now_s();
    if (ctx && n > 0) {
        void *p = NULL;
        hipSetDevice(0);
        hipMalloc(&p, 1 << 20);
        hipMemset(p, 0, 1 << 20);
        hipDeviceSynchronize();
        hipFree(p);
    }
    const double t2 = now_s();
    if (sleep_ms > 0) usleep((useconds_t)sleep_ms * 1000u);
    if (thread) {
        pthread_t th;
        if (pthread_create(&th, NULL, noop, NULL) == 0) pthread_join(th, NULL);
    }
    if (pool > 0) {  /* pool=N: N threads busy for 2 ms each, joined (the CLI writer's shape) */
        pthread_t th[64];
        int ok[64] = {0};
        if (pool > 64) pool = 64;
        for (int i = 0; i < pool; i++) ok[i] = pthread_create(&th[i], NULL, spin, NULL) == 0;
        for (int i = 0; i < pool; i++)
            if (ok[i]) pthread_join(th[i], NULL);
    }
    fprintf(stderr, "hipinit_probe: devices %d count %.3f ctx %.3f\n", n, t1 - t0, t2 - t1);
    fprintf(stderr, "hipinit_probe clock: main_entry %.6f main_return %.6f\n", t0, now_s());
    fflush(stderr);
    if (fast) _exit(0);
    return 0;
}
