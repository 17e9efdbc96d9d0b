/*
 * oracle.h -- CPU restatement of rik1599/SimplexOnCuda's dense two-phase simplex.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker (or as the timed
 * CPU baseline).  The product (libsimplex_hip.so) never links or calls it.
 *
 * Orientation: the reference keeps the TRANSPOSED tableau (one pitched row per variable,
 * one column per constraint; tabular.cu:25-39).  This restatement keeps the textbook
 * orientation, which is what the HIP product stores in HBM:
 *     T[i][j], i in [0,m) constraint rows, j in [0,N) columns, row stride ld
 *     column 0 = RHS b, column v+1 = variable v (x: 0..n-1, slack n..n+m-1,
 *     artificial n+m..n+2m-1);  N = N1 = 1+n+2m (phase 1) or N2 = 1+n+m (phase 2)
 *     d[0..N)   objective row ("costsVector"), d[0] = objective value
 * The arithmetic is element-for-element the reference's.
 *
 * Parity pins (see tests/test_oracle.py): the 36 published pivot counts harvested from
 * data/measures/<gpu>/benchmark_<n>_<m>.txt line counts, hand-traced example answers,
 * and SciPy/HiGHS objective values computed in the build container.
 */
#ifndef SIMPLEX_ORACLE_H
#define SIMPLEX_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes: twoPhaseMethod.h:5-8 and solver.cu:77 */
#define ORC_FEASIBLE 0
#define ORC_INFEASIBLE (-1)
#define ORC_UNBOUNDED (-2)
#define ORC_DEGENERATE (-3)
#define ORC_NOT_ENDED (-10)
#define ORC_PIVOT_CAP (-11) /* opt-in iteration cap reached (not a reference status) */

/* host C runtime rand() flavours used by srand/rand in problem.cu:63-67 */
#define ORC_RAND_MSVC 0
#define ORC_RAND_GLIBC 1

/* ---- generator (problem.cu:49-126, generator.cu:9-32) ---- */
void orc_crt_rand(unsigned seed, int kind, int count, uint32_t *out);
void orc_xorwow_draws(uint64_t seed, uint64_t offset, int64_t count, uint32_t *out);
/* contract: 1 = nvcc default fp contraction (fmaf / fma), 0 = separate mul + add */
void orc_generate_problem(int n, int m, unsigned seed, int lo, int hi, int rand_kind, int contract,
                          double *A_colmajor, double *b, double *c);

/* ---- epsilon argmin (reduction.cu:10-104) ---- */
int64_t orc_argmin(const double *v, int64_t L, double *vmin);
/* stage 1 on one 512-element tile: elements v[0..len) carry global indices gidx0.. */
void orc_argmin_tile(const double *v, int64_t len, int64_t gidx0, double *pv, int64_t *pi);
/* stage 2 over B (<= 1024) tile winners, reference pass-2 tree (reduction.cu:239-241) */
int64_t orc_argmin_pass2(const double *pv, const int64_t *pi, int64_t B, double *vmin);

/* ---- tableau ---- */
void orc_build_phase1(int n, int m, const double *A_colmajor, const double *b,
                      double *T, int64_t ld, double *d, int *base);
/* blocked deterministic objective GEMV (gaussian.cu:132-162 semantics, fixed order):
 * partial[k][j] = fma-chain over rows of 512-row block k, d[j] -= sum_k partial[k][j] */
void orc_gemv_partials(const double *T, int64_t rows, int64_t N, int64_t ld, const double *coef,
                       double *partials);
void orc_gemv_apply(double *d, int64_t N, const double *partials, int64_t nblk);
void orc_update_objective(const double *T, int64_t m, int64_t N, int64_t ld, const int *base, double *d);

/* ratio vector entry (reduction.cu:106-114) */
double orc_ratio(double b, double a);

/* rank-1 update of rows [0,rows) of a row block plus (optionally) d.
 * prow = pre-update pivot row, colE[i] = pre-update entering-column entry of local row i,
 * r_local = pivot row index inside this block or -1, p = pivot, d_e = entering reduced cost */
/* host threads of orc_apply_update (default 1; the arithmetic is per element, so the result does
   not depend on it) */
void orc_set_threads(int n);
void orc_apply_update(double *T, int64_t rows, int64_t N, int64_t ld, double *d, const double *prow,
                      const double *colE, int64_t r_local, double p, double d_e);

/* one pivot (solver.cu:78-126). Returns ORC_NOT_ENDED / ORC_FEASIBLE / ORC_UNBOUNDED */
int orc_pivot(double *T, int64_t m, int64_t N, int64_t ld, double *d, int *base, int64_t *e_out,
              int64_t *r_out);
/* pivot loop (solver.cu:128-149); max_pivots < 0 = no cap (parity mode) */
int orc_solve(double *T, int64_t m, int64_t N, int64_t ld, double *d, int *base, int64_t max_pivots,
              int64_t *pivots);

/* full two-phase method (twoPhaseMethod.cu:225-435). pivots[2] = P1/P2 counts. */
int orc_two_phase(int n, int m, const double *A_colmajor, const double *b, const double *c,
                  int64_t max_pivots, double *x, double *opt, int *base_out, int64_t *pivots,
                  double *phase1_value);

/* problem text file (problem.cu:20-47). Returns 0 on success. A is column-major. */
int orc_read_problem_header(const char *path, int *n, int *m);
int orc_read_problem(const char *path, double *A_colmajor, double *b, double *c);

#ifdef __cplusplus
}
#endif
#endif
