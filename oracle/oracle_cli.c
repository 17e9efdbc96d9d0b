#define _POSIX_C_SOURCE 199309L
/* oracle_cli.c -- command-line driver of the CPU oracle (TEST INFRASTRUCTURE).
 *   oracle_cli gen  <n> <m> <seed> [lo hi rand contract max_pivots]
 *   oracle_cli file <path>
 * Prints: status P1 P2 opt phase1_value seconds  (one line, space separated) */
#include "oracle.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s gen n m seed [lo hi rand contract max_pivots] | file path\n", argv[0]);
        return 2;
    }
    int n, m;
    double *A, *b, *c;
    long long cap = -1;
    if (!strcmp(argv[1], "gen")) {
        n = atoi(argv[2]);
        m = atoi(argv[3]);
        unsigned seed = (unsigned)strtoul(argv[4], NULL, 10);
        int lo = argc > 5 ? atoi(argv[5]) : 1, hi = argc > 6 ? atoi(argv[6]) : 100;
        int rk = argc > 7 ? atoi(argv[7]) : ORC_RAND_MSVC, ct = argc > 8 ? atoi(argv[8]) : 1;
        cap = argc > 9 ? atoll(argv[9]) : -1;
        A = malloc(sizeof(double) * (size_t)n * m);
        b = malloc(sizeof(double) * m);
        c = malloc(sizeof(double) * n);
        orc_generate_problem(n, m, seed, lo, hi, rk, ct, A, b, c);
    } else {
        if (orc_read_problem_header(argv[2], &n, &m)) return 1;
        A = malloc(sizeof(double) * (size_t)n * m);
        b = malloc(sizeof(double) * m);
        c = malloc(sizeof(double) * n);
        if (orc_read_problem(argv[2], A, b, c)) return 1;
    }
    double *x = malloc(sizeof(double) * n), opt = 0, p1v = 0;
    int *base = malloc(sizeof(int) * m);
    int64_t piv[2];
    double t0 = now();
    int st = orc_two_phase(n, m, A, b, c, cap, x, &opt, base, piv, &p1v);
    double t1 = now();
    printf("%d %lld %lld %.17g %.17g %.3f\n", st, (long long)piv[0], (long long)piv[1], opt, p1v, t1 - t0);
    free(A);
    free(b);
    free(c);
    free(x);
    free(base);
    return 0;
}
