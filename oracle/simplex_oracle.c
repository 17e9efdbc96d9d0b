/*
 * simplex_oracle.c -- serial CPU restatement of rik1599/SimplexOnCuda (TEST INFRASTRUCTURE).
 *
 * This file is the checker for the HIP product and the "port" CPU baseline timed by
 * bench.py.  It is never linked into the product.  Each function cites the reference
 * file:line whose behaviour it restates.  Compiled with -ffp-contract=off: every fused
 * multiply-add in the reference is written here as an explicit fma().
 *
 * Third-party arithmetic restated here (absent from /root/reference):
 *   - cuRAND XORWOW (curand_kernel.h: curand_init / curand / curand_uniform), used by
 *     generator.cu:13-18,27-30.  Published algorithm: Marsaglia xorwow with cuRAND's
 *     seed scrambling; pinned indirectly by the published pivot counts (tests/golden).
 *   - the host CRT rand() (problem.cu:63-67): MSVC LCG or glibc TYPE_3 additive.
 */
#include "oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define EPS 1e-9
#define TILE 512          /* THREADS in reduction.cu:6 */
#define WARP 32           /* CUDA warpSize */
#define MAXGRID 1024      /* BL(N) cap, reduction.cu:7 */
#define GEMV_BLOCK 512    /* fixed summation block of the objective GEMV (see header) */

/* macro.h:28-42 -- compare(x, y, eps=1e-9) */
static inline int cmp_eps(double x, double y) {
    if (fabs(x - y) < EPS) return 0;
    if (x < y) return -1;
    return 1;
}

/* ======================= generator ======================= */

/* problem.cu:63-67 srand(seed); rand() x3 */
void orc_crt_rand(unsigned seed, int kind, int count, uint32_t *out) {
    if (kind == ORC_RAND_MSVC) {
        uint32_t h = seed;
        for (int k = 0; k < count; ++k) {
            h = h * 214013u + 2531011u;
            out[k] = (h >> 16) & 0x7fffu;
        }
        return;
    }
    /* glibc random_r TYPE_3 (r = 3, deg 31, sep 3) */
    int32_t r[34 + 344 + 64];
    int total = 34 + 310 + count;
    int32_t *rr = r;
    int32_t *heap = NULL;
    if (total > (int)(sizeof(r) / sizeof(r[0]))) {
        heap = (int32_t *)malloc(sizeof(int32_t) * (size_t)total);
        rr = heap;
    }
    if (seed == 0) seed = 1;
    rr[0] = (int32_t)seed;
    for (int i = 1; i < 31; ++i) {
        int64_t v = (16807LL * rr[i - 1]) % 2147483647LL;
        if (v < 0) v += 2147483647LL;
        rr[i] = (int32_t)v;
    }
    for (int i = 31; i < 34; ++i) rr[i] = rr[i - 31];
    for (int i = 34; i < total; ++i) rr[i] = (int32_t)((uint32_t)rr[i - 31] + (uint32_t)rr[i - 3]);
    for (int k = 0; k < count; ++k) out[k] = ((uint32_t)rr[344 + k]) >> 1;
    free(heap);
}

/* curand_init(seed, 0, 0) state + curand() step (XORWOW) */
typedef struct {
    uint32_t d;
    uint32_t v[5];
} xorwow_t;

static void xorwow_init(xorwow_t *s, uint64_t seed) {
    uint32_t s0 = ((uint32_t)seed) ^ 0xaad26b49u;
    uint32_t s1 = ((uint32_t)(seed >> 32)) ^ 0xf7dcefddu;
    uint32_t t0 = 1099087573u * s0;
    uint32_t t1 = 2591861531u * s1;
    s->d = 6615241u + t1 + t0;
    s->v[0] = 123456789u + t0;
    s->v[1] = 362436069u ^ t0;
    s->v[2] = 521288629u + t1;
    s->v[3] = 88675123u ^ t1;
    s->v[4] = 5783321u + t0;
}

static inline uint32_t xorwow_next(xorwow_t *s) {
    uint32_t t = s->v[0] ^ (s->v[0] >> 2);
    s->v[0] = s->v[1];
    s->v[1] = s->v[2];
    s->v[2] = s->v[3];
    s->v[3] = s->v[4];
    s->v[4] = (s->v[4] ^ (s->v[4] << 4)) ^ (t ^ (t << 1));
    s->d += 362437u;
    return s->v[4] + s->d;
}

/* draws #offset .. #offset+count-1 of the subsequence-0 stream of `seed`.
 * curand_init(seed, 0, k) positions the state exactly k draws in (generator.cu:15,29). */
void orc_xorwow_draws(uint64_t seed, uint64_t offset, int64_t count, uint32_t *out) {
    xorwow_t s;
    xorwow_init(&s, seed);
    for (uint64_t k = 0; k < offset; ++k) (void)xorwow_next(&s);
    for (int64_t k = 0; k < count; ++k) out[k] = xorwow_next(&s);
}

/* curand_uniform: x * CURAND_2POW32_INV + CURAND_2POW32_INV/2 (float) */
static inline float uniform01(uint32_t x, int contract) {
    const float inv = 2.3283064e-10f;
    const float half = inv / 2.0f;
    return contract ? fmaf((float)x, inv, half) : (float)x * inv + half;
}

/* generator.cu:18,30: (curand_uniform * (max - min)) + min, promoted to double */
static inline double scale_value(float u, double lo, double hi, int contract) {
    return contract ? fma((double)u, hi - lo, lo) : (double)u * (hi - lo) + lo;
}

/* problem.cu:49-126 + generator.cu:9-32.
 * A(i,j): thread i (constraint) does curand_init(sA, 0, i*n) and draws j = 0..n-1, so the
 * row-major flattening of A is one sequential stream.  b_i, c_j: draw #i / #j. */
void orc_generate_problem(int n, int m, unsigned seed, int lo, int hi, int rand_kind, int contract,
                          double *A_colmajor, double *b, double *c) {
    uint32_t sd[3];
    orc_crt_rand(seed, rand_kind, 3, sd);
    const uint32_t sB = sd[0], sC = sd[1], sA = sd[2];
    const double dlo = (double)lo, dhi = (double)hi;
    xorwow_t s;
    xorwow_init(&s, sB);
    for (int i = 0; i < m; ++i) b[i] = scale_value(uniform01(xorwow_next(&s), contract), dlo, dhi, contract);
    xorwow_init(&s, sC);
    for (int j = 0; j < n; ++j) c[j] = scale_value(uniform01(xorwow_next(&s), contract), dlo, dhi, contract);
    xorwow_init(&s, sA);
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < n; ++j)
            A_colmajor[(int64_t)j * m + i] = scale_value(uniform01(xorwow_next(&s), contract), dlo, dhi, contract);
}

/* ======================= epsilon argmin ======================= */

typedef struct {
    double v;
    int64_t i;
} vi_t;

/* warpReduceMin (reduction.cu:10-22): lane l <- combine(lane l, lane l+off) for off=16..1;
 * the shuffled-in value replaces the lane's only if compare(shfl, own) < 0. */
static vi_t warp32(vi_t *l) {
    for (int off = WARP / 2; off > 0; off >>= 1)
        for (int k = 0; k + off < WARP; ++k)
            if (cmp_eps(l[k + off].v, l[k].v) < 0) l[k] = l[k + off];
    return l[0];
}

/* blockReduceMin (reduction.cu:24-49) over `threads` per-thread values */
static vi_t block_reduce(vi_t *th, int threads) {
    vi_t win[WARP];
    int nw = threads / WARP;
    for (int w = 0; w < WARP; ++w) {
        win[w].v = DBL_MAX;
        win[w].i = -1;
    }
    for (int w = 0; w < nw; ++w) win[w] = warp32(th + w * WARP);
    return warp32(win);
}

void orc_argmin_tile(const double *v, int64_t len, int64_t gidx0, double *pv, int64_t *pi) {
    vi_t th[TILE];
    for (int t = 0; t < TILE; ++t) {
        th[t].v = DBL_MAX;
        th[t].i = -1;
        if (t < len && cmp_eps(v[t], DBL_MAX) < 0) {
            th[t].v = v[t];
            th[t].i = gidx0 + t;
        }
    }
    vi_t r = block_reduce(th, TILE);
    *pv = r.v;
    *pi = r.i;
}

/* deviceReduceKernel<false><<<1,1024>>> (reduction.cu:51-80, 239-241) */
int64_t orc_argmin_pass2(const double *pv, const int64_t *pi, int64_t B, double *vmin) {
    vi_t th[MAXGRID];
    for (int t = 0; t < MAXGRID; ++t) {
        th[t].v = DBL_MAX;
        th[t].i = -1;
        for (int64_t k = t; k < B; k += MAXGRID)
            if (cmp_eps(pv[k], th[t].v) < 0) {
                th[t].v = pv[k];
                th[t].i = pi[k];
            }
    }
    vi_t r = block_reduce(th, MAXGRID);
    if (vmin) *vmin = r.v;
    return r.i;
}

/* minElement(g_vet, size, &idx) (reduction.cu:82-104): pass 1 with BL(size) blocks of 512
 * threads (grid-stride when size > 512*1024), then pass 2 if BL(size) > 1. */
int64_t orc_argmin(const double *v, int64_t L, double *vmin) {
    int64_t grid = (L + TILE - 1) / TILE;
    if (grid > MAXGRID) grid = MAXGRID;
    if (grid < 1) grid = 1;
    double *pv = (double *)malloc(sizeof(double) * (size_t)grid);
    int64_t *pi = (int64_t *)malloc(sizeof(int64_t) * (size_t)grid);
    vi_t th[TILE];
    for (int64_t b = 0; b < grid; ++b) {
        for (int t = 0; t < TILE; ++t) {
            th[t].v = DBL_MAX;
            th[t].i = -1;
            for (int64_t i = b * TILE + t; i < L; i += TILE * grid)
                if (cmp_eps(v[i], th[t].v) < 0) {
                    th[t].v = v[i];
                    th[t].i = i;
                }
        }
        vi_t r = block_reduce(th, TILE);
        pv[b] = r.v;
        pi[b] = r.i;
    }
    int64_t idx;
    if (grid > 1) {
        idx = orc_argmin_pass2(pv, pi, grid, vmin);
    } else {
        idx = pi[0];
        if (vmin) *vmin = pv[0];
    }
    free(pv);
    free(pi);
    return idx;
}

/* ======================= tableau ======================= */

/* twoPhaseMethod.cu:145-200 (fillTableu) + checkColumns/negateColumn 86-111, in row-major */
void orc_build_phase1(int n, int m, const double *A_colmajor, const double *b, double *T, int64_t ld,
                      double *d, int *base) {
    const int64_t N1 = 1 + (int64_t)n + 2 * (int64_t)m;
    for (int i = 0; i < m; ++i) {
        double *row = T + (int64_t)i * ld;
        memset(row, 0, sizeof(double) * (size_t)ld);
        row[0] = b[i];
        for (int j = 0; j < n; ++j) row[1 + j] = A_colmajor[(int64_t)j * m + i];
        row[1 + n + i] = 1.0;       /* slack (fillMatrix, :36) */
        row[1 + n + m + i] = 1.0;   /* artificial (fillMatrix, :37) */
        base[i] = n + m + i;        /* fillBaseVector (:44-52) */
    }
    for (int64_t j = 0; j < N1; ++j) d[j] = (j <= (int64_t)n + m) ? 0.0 : 1.0; /* :152-157 */
    /* checkColumns: every constraint with compare(b_i) < 0 is negated across ALL its
     * entries, slack and artificial included (the reference quirk). */
    for (int i = 0; i < m; ++i) {
        double *row = T + (int64_t)i * ld;
        if (cmp_eps(row[0], 0.0) < 0)
            for (int64_t j = 0; j < N1; ++j) row[j] = -row[j];
    }
}

void orc_gemv_partials(const double *T, int64_t rows, int64_t N, int64_t ld, const double *coef,
                       double *partials) {
    int64_t nblk = (rows + GEMV_BLOCK - 1) / GEMV_BLOCK;
    for (int64_t k = 0; k < nblk; ++k) {
        double *p = partials + k * N;
        for (int64_t j = 0; j < N; ++j) p[j] = 0.0;
        int64_t i1 = (k + 1) * GEMV_BLOCK < rows ? (k + 1) * GEMV_BLOCK : rows;
        for (int64_t i = k * GEMV_BLOCK; i < i1; ++i) {
            const double *row = T + i * ld;
            const double ci = coef[i];
            for (int64_t j = 0; j < N; ++j) p[j] = fma(row[j], ci, p[j]);
        }
    }
}

void orc_gemv_apply(double *d, int64_t N, const double *partials, int64_t nblk) {
    for (int64_t j = 0; j < N; ++j) {
        double s = partials[j];
        for (int64_t k = 1; k < nblk; ++k) s = s + partials[k * N + j];
        d[j] = d[j] - s;
    }
}

/* updateObjectiveFunction (gaussian.cu:132-162): coef[i] = d[1+base[i]] snapshot, then
 * d[j] -= sum_i T[i][j]*coef[i] for every column j (RHS column included). */
void orc_update_objective(const double *T, int64_t m, int64_t N, int64_t ld, const int *base, double *d) {
    double *coef = (double *)malloc(sizeof(double) * (size_t)m);
    for (int64_t i = 0; i < m; ++i) coef[i] = d[1 + base[i]];
    int64_t nblk = (m + GEMV_BLOCK - 1) / GEMV_BLOCK;
    double *part = (double *)malloc(sizeof(double) * (size_t)(nblk * N));
    orc_gemv_partials(T, m, N, ld, coef, part);
    orc_gemv_apply(d, N, part, nblk);
    free(part);
    free(coef);
}

/* createIndicatorsVector (reduction.cu:106-114) */
double orc_ratio(double b, double a) { return cmp_eps(a, 0.0) > 0 ? b / a : DBL_MAX; }

/* updateContraintsMatrix + updateCostsVector (solver.cu:34-56):
 *   row r:      T[r][j] / p
 *   other rows: fma(-(a_ie/p), T_old[r][j], T[i][j])
 *   objective:  fma(-(d_e/p),  T_old[r][j], d[j]) */
static void update_rows(double *T, int64_t i0, int64_t i1, int64_t N, int64_t ld, const double *prow,
                        const double *colE, int64_t r_local, double p) {
    for (int64_t i = i0; i < i1; ++i) {
        double *row = T + i * ld;
        if (i == r_local) {
            for (int64_t j = 0; j < N; ++j) row[j] = prow[j] / p;
        } else {
            const double f = -colE[i] / p;
            for (int64_t j = 0; j < N; ++j) row[j] = fma(f, prow[j], row[j]);
        }
    }
}

/* Rows may be updated by several host threads (orc_set_threads, default 1): every element still
   receives exactly the one operation above, so the result does not depend on the thread count.
   Used only to make the long full-size pins (tests/golden/scripts/make_long_pins.py) affordable;
   the timed CPU baseline runs with one thread. */
static int g_threads = 1;
void orc_set_threads(int n) { g_threads = n < 1 ? 1 : n > 64 ? 64 : n; }

struct upd_job {
    double *T;
    int64_t i0, i1, N, ld, r_local;
    const double *prow, *colE;
    double p;
};
static void *upd_thread(void *a) {
    const struct upd_job *j = (const struct upd_job *)a;
    update_rows(j->T, j->i0, j->i1, j->N, j->ld, j->prow, j->colE, j->r_local, j->p);
    return NULL;
}

void orc_apply_update(double *T, int64_t rows, int64_t N, int64_t ld, double *d, const double *prow,
                      const double *colE, int64_t r_local, double p, double d_e) {
    const int nt = (rows * N >= ((int64_t)1 << 22)) ? g_threads : 1;
    if (nt <= 1) {
        update_rows(T, 0, rows, N, ld, prow, colE, r_local, p);
    } else {
        pthread_t th[64];
        int started[64];
        struct upd_job job[64];
        for (int k = 0; k < nt; ++k) {
            job[k] = (struct upd_job){T, rows * k / nt, rows * (k + 1) / nt, N, ld, r_local, prow, colE, p};
            started[k] = pthread_create(&th[k], NULL, upd_thread, &job[k]) == 0;
            if (!started[k]) upd_thread(&job[k]);
        }
        for (int k = 0; k < nt; ++k)
            if (started[k]) pthread_join(th[k], NULL);
    }
    if (d) {
        const double f = -d_e / p;
        for (int64_t j = 0; j < N; ++j) d[j] = fma(f, prow[j], d[j]);
    }
}

/* one iteration of solve (solver.cu:78-126) */
int orc_pivot(double *T, int64_t m, int64_t N, int64_t ld, double *d, int *base, int64_t *e_out,
              int64_t *r_out) {
    double dmin;
    int64_t e = orc_argmin(d + 1, N - 1, &dmin); /* :87 */
    if (e_out) *e_out = e;
    if (r_out) *r_out = -1;
    if (!(cmp_eps(dmin, 0.0) < 0)) return ORC_FEASIBLE; /* :88, :119-125 */
    double *colE = (double *)malloc(sizeof(double) * (size_t)m);
    double *ratio = (double *)malloc(sizeof(double) * (size_t)m);
    int any = 0;
    for (int64_t i = 0; i < m; ++i) {
        colE[i] = T[i * ld + 1 + e];
        if (colE[i] >= EPS) any = 1; /* isLessOrEqualThanZero: compare(max) <= 0 (:96) */
    }
    if (!any) {
        free(colE);
        free(ratio);
        return ORC_UNBOUNDED;
    }
    for (int64_t i = 0; i < m; ++i) ratio[i] = orc_ratio(T[i * ld], colE[i]);
    int64_t r = orc_argmin(ratio, m, NULL); /* :104 */
    if (r_out) *r_out = r;
    base[r] = (int)e; /* :105 */
    double *prow = (double *)malloc(sizeof(double) * (size_t)N);
    memcpy(prow, T + r * ld, sizeof(double) * (size_t)N);
    const double p = prow[1 + e];
    orc_apply_update(T, m, N, ld, d, prow, colE, r, p, dmin);
    free(prow);
    free(colE);
    free(ratio);
    return ORC_NOT_ENDED;
}

/* solve(tabular_t*, int*) (solver.cu:128-149) */
int orc_solve(double *T, int64_t m, int64_t N, int64_t ld, double *d, int *base, int64_t max_pivots,
              int64_t *pivots) {
    int64_t k = 0;
    int st;
    for (;;) {
        if (max_pivots >= 0 && k >= max_pivots) {
            st = ORC_PIVOT_CAP;
            break;
        }
        st = orc_pivot(T, m, N, ld, d, base, NULL, NULL);
        if (st != ORC_NOT_ENDED) break;
        ++k;
    }
    if (pivots) *pivots = k;
    return st;
}

/* the last orc_two_phase call's final objective row: phase 2's (width 1+n+m) when phase 1 ended
   feasible, else phase 1's (width 1+n+2m) -- what simplex_last_objective_row returns */
static double *g_last_d = NULL;
static int64_t g_last_n = 0;
static void keep_last_d(const double *d, int64_t n) {
    free(g_last_d);
    g_last_d = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    memcpy(g_last_d, d, sizeof(double) * (size_t)n);
    g_last_n = n;
}
int64_t orc_last_objective_row(double *out, int64_t cap) {
    for (int64_t j = 0; out && j < g_last_n && j < cap; ++j) out[j] = g_last_d[j];
    return g_last_n;
}

/* twoPhaseMethod (twoPhaseMethod.cu:225-435) */
int orc_two_phase(int n, int m, const double *A_colmajor, const double *b, const double *c,
                  int64_t max_pivots, double *x, double *opt, int *base_out, int64_t *pivots,
                  double *phase1_value) {
    const int64_t N1 = 1 + (int64_t)n + 2 * (int64_t)m;
    const int64_t N2 = 1 + (int64_t)n + (int64_t)m;
    const int64_t ld = N1;
    double *T = (double *)malloc(sizeof(double) * (size_t)(ld * m));
    double *d = (double *)malloc(sizeof(double) * (size_t)N1);
    int *base = (int *)malloc(sizeof(int) * (size_t)m);
    int64_t p1 = 0, p2 = 0;
    int status;

    orc_build_phase1(n, m, A_colmajor, b, T, ld, d, base);
    orc_update_objective(T, m, N1, ld, base, d);              /* gauss1, :247 */
    int st1 = orc_solve(T, m, N1, ld, d, base, max_pivots, &p1); /* :258, status ignored */
    if (phase1_value) *phase1_value = d[0];
    if (st1 == ORC_PIVOT_CAP) {
        status = ORC_PIVOT_CAP;
    } else if (cmp_eps(d[0], 0.0) < 0) { /* :265-268 */
        status = ORC_INFEASIBLE;
    } else {
        status = ORC_FEASIBLE;
        for (int i = 0; i < m; ++i) /* checkDegeneracy :206-223 */
            if (base[i] >= n + m && base[i] < n + 2 * m) status = ORC_DEGENERATE;
    }
    if (status != ORC_FEASIBLE) keep_last_d(d, N1);
    if (status == ORC_FEASIBLE) {
        /* phase2 (:285-356): drop artificial columns, d[1..n] = -c, slacks 0, d[0] kept */
        for (int j = 0; j < n; ++j) d[1 + j] = -c[j];
        for (int j = 0; j < m; ++j) d[1 + n + j] = 0.0;
        orc_update_objective(T, m, N2, ld, base, d); /* gauss2, :337 */
        int64_t cap2 = max_pivots < 0 ? -1 : max_pivots;
        status = orc_solve(T, m, N2, ld, d, base, cap2, &p2);
        keep_last_d(d, N2);
        if (status == ORC_FEASIBLE) {
            /* getSolutionHost (:370-383) */
            if (opt) *opt = d[0];
            if (x) {
                for (int j = 0; j < n; ++j) x[j] = 0.0;
                for (int i = 0; i < m; ++i)
                    if (base[i] < n) x[base[i]] = T[(int64_t)i * ld];
            }
        }
    }
    if (base_out) memcpy(base_out, base, sizeof(int) * (size_t)m);
    if (pivots) {
        pivots[0] = p1;
        pivots[1] = p2;
    }
    free(T);
    free(d);
    free(base);
    return status;
}

/* readProblemFromFile (problem.cu:20-47): "n m", c[n], then m lines of A-row and b_i */
int orc_read_problem_header(const char *path, int *n, int *m) {
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    int ok = fscanf(f, "%d %d", n, m) == 2;
    fclose(f);
    return ok ? 0 : -1;
}

int orc_read_problem(const char *path, double *A_colmajor, double *b, double *c) {
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    int n = 0, m = 0;
    if (fscanf(f, "%d %d", &n, &m) != 2) {
        fclose(f);
        return -1;
    }
    for (int j = 0; j < n; ++j)
        if (fscanf(f, "%lf", &c[j]) != 1) goto fail;
    for (int i = 0; i < m; ++i) {
        for (int j = 0; j < n; ++j)
            if (fscanf(f, "%lf", &A_colmajor[(int64_t)j * m + i]) != 1) goto fail;
        if (fscanf(f, "%lf", &b[i]) != 1) goto fail;
    }
    fclose(f);
    return 0;
fail:
    fclose(f);
    return -1;
}
