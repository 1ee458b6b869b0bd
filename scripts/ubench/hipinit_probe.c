/* Floor of a HIP command-line program: load the runtime, count the devices
 * (HIP start-up), optionally touch device 0 (context), then exit normally or
 * by _exit (no runtime teardown).  Usage: hipinit_probe [ctx] [fast] */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int main(int argc, char **argv)
{
    int ctx = 0, fast = 0;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "ctx")) ctx = 1;
        if (!strcmp(argv[i], "fast")) fast = 1;
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
    fprintf(stderr, "hipinit_probe: devices %d count %.3f ctx %.3f\n", n, t1 - t0, t2 - t1);
    if (fast) _exit(0);
    return 0;
}
