/* oracle/orc_main.c -- TEST INFRASTRUCTURE ONLY.  Command-line driver for the
 * CPU restatement, same flags and defaults as the reference
 * (sources/main_MIDASPOM.c:66-118) plus -t <threads>.  Prints only the
 * "Total log-likelihood=" line (:425); the posterior file layout is :427-436. */
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

#include "spom_oracle.h"

int main(int argc, char **argv)
{
    double m = 400, d = 100, lo = 0, hi = 1;
    float p = 0.5f;
    const char *in = "input.txt", *out = "posterior.txt";
    unsigned s = 101, threads = 1;
    int ch;
    while ((ch = getopt(argc, argv, "m:p:d:i:o:s:l:u:t:")) != -1) {
        switch (ch) {
        case 'm': m = atof(optarg); break;
        case 'p': p = (float)atof(optarg); break;
        case 'd': d = atof(optarg); break;
        case 'i': in = optarg; break;
        case 'o': out = optarg; break;
        case 's': s = (unsigned)atoi(optarg); break;
        case 'l': lo = atof(optarg); break;
        case 'u': hi = atof(optarg); break;
        case 't': threads = (unsigned)atoi(optarg); break;
        default: return 1;
        }
    }
    double ltot;
    int rc = orc_run(in, out, m, p, d, s, lo, hi, threads, NULL, &ltot);
    if (rc) { fprintf(stderr, "oracle failed: %d\n", rc); return 2; }
    printf("Total log-likelihood=%.5lf\n", ltot);
    return 0;
}
