// sx_common.hpp -- shared host/device definitions of the MI355X simplex engine.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

// Status codes: twoPhaseMethod.h:5-8 (reference), solver.cu:77 (NOT_ENDED), plus two
// engine-only codes that the reference has no equivalent for.
#define SX_FEASIBLE 0
#define SX_INFEASIBLE (-1)
#define SX_UNBOUNDED (-2)
#define SX_DEGENERATE (-3)
#define SX_NOT_ENDED (-10)
#define SX_PIVOT_CAP (-11)     // opt-in pivot budget reached (off in parity mode)
#define SX_NUMERIC_FAIL (-12)  // ratio argmin returned no row although a pivot is eligible

#define SX_TILE 512     // argmin tile = reference THREADS (reduction.cu:6)
#define SX_EPS 1e-9     // macro.h:28

// One 512-element argmin tile winner, plus "this tile has an entry >= eps" for the
// unbounded test.  16 bytes: moved as raw bytes by the tile allgather.
struct __attribute__((aligned(16))) TilePart {
    double v;
    int idx;
    int elig;
};

// Per-shard pivot state, resident in device memory (never read by the host inside a
// batch of pivots).
struct __attribute__((aligned(16))) DevState {
    int status;            // SX_NOT_ENDED while the phase runs
    int e;                 // entering variable of the current pivot (column e+1)
    int r;                 // leaving row (global) of the current pivot; after the update its
                           // new values sit in rnew[pivots & 1] until the next update writes
                           // them back (the row is read in place as the pivot row meanwhile)
    int r_prev;            // leaving row of the previous pivot
    double dmin;           // reduced cost of the entering variable (d[e+1] before update)
    long long pivots;      // pivots applied in this phase
    long long max_pivots;  // < 0: no cap (reference behaviour)
    int e_next;            // entering argmin of the updated objective row (next pivot)
    unsigned ticket;       // arrival counter of the ratio/select hand-off (zero between launches)
    double dmin_next;      // its value
    unsigned ticket_d;     // arrival counter of the objective-row blocks of the update
    int touched;           // this shard's rows the current update sweeps (rows with a nonzero factor)
    int touched_pairs;     // column pairs of the current pivot row holding a nonzero (swept columns)
    int pad1;
};

// tile_cnt[t] of a ratio tile: the number of listed rows, plus SX_TILE_WIDE when a listed
// row's entry is too large for the factor -a/p to be finite with p >= eps
#define SX_TILE_WIDE 0x40000000
#define SX_TILE_COUNT(x) ((x) & (SX_TILE_WIDE - 1))

// TilePart.elig packs "any entry >= eps" (bit 0) and the tile's count of nonzero
// entering-column entries (bits 1..)
#define SX_ELIG(x) ((x) & 1)
#define SX_NNZ(x) ((x) >> 1)

// Error convention of the reference (error.cu:5-12): print "<msg> in <file> at line <n>"
// and exit(EXIT_FAILURE).
void sx_handle_error(hipError_t err, const char *file, int line);
#define SX_HIP(call) sx_handle_error((call), __FILE__, __LINE__)
void sx_fatal(const char *msg, const char *file, int line);
#define SX_FATAL(msg) sx_fatal((msg), __FILE__, __LINE__)

// Logical vs stored tableau columns.  In phase 1 every artificial column n+m+k starts equal
// to its slack column n+k (both unit vectors, both negated by the b<0 quirk) and receives
// exactly the same IEEE operations at every pivot, so the two stay bit-identical: only
// Ns = 1+n+m columns are stored and logical column j >= art0 reads stored column j - shift.
struct Cols {
    int N;      // logical columns of the phase (reference width: 1+n+2m or 1+n+m)
    int Ns;     // stored columns (swept by the update)
    int art0;   // first aliased logical column, or INT_MAX
    int shift;  // alias distance (m)
    __host__ __device__ __forceinline__ int map(int j) const { return j >= art0 ? j - shift : j; }
};

// ---- kernel launchers (sx_kernels.hip) ----
struct UpdateCfg {
    int rows_per_block;  // 1, 2, 4 or 8
    int snake;           // alternate the sweep direction every pivot
    int sc1;             // write-through (sc1) tableau stores
    int skip_zero;       // skip rows whose factor is exactly zero (only when bit-exact: no -0.0 in T)
    int one_shot;        // 1: one block per (512 columns, RB rows); 0: resident blocks sweep the row list
};

int sx_enter_blocks(int L);
void sx_launch_enter(const double *d, int L, TilePart *parts, DevState *st, hipStream_t s);
void sx_launch_ratio_select(const double *T, int rows, int row0, size_t ld, TilePart *tiles_local, double *colE,
                            DevState *st, int *base, const double *rnew, size_t rnew_stride, bool select,
                            double *slots, size_t slot_stride, Cols c, int *rowlist, int *tile_cnt, int skip_zero,
                            hipStream_t s);
void sx_launch_select_gathered(const double *slots, size_t slot_stride, int B2, int *base, DevState *st,
                               int tile0, int nslots, hipStream_t s);
void sx_launch_select_row(const double *T, int rows, int row0, size_t ld, Cols c, const TilePart *tiles_all, int B2,
                          double *prow_out, int *base, DevState *st, const double *rnew, size_t rnew_stride,
                          int tile0, int slots, hipStream_t s);
void sx_launch_update(double *T, int rows, int row0, size_t ld, Cols c, double *d, const double *prow_buf,
                      size_t prow_stride, const double *colE, DevState *st, double *rnew, size_t rnew_stride,
                      TilePart *enter_parts, const int *rowlist, const int *tile_cnt, UpdateCfg cfg, hipStream_t s);
void sx_set_update_waves(float w);  // resident-grid multiple of the update's row sweep (default 2)
void sx_launch_flush_row(double *T, int rows, int row0, size_t ld, int Ns, const double *rnew, size_t rnew_stride,
                         const DevState *st, hipStream_t s);
void sx_launch_sum_rows(double *out, const double *const *srcs, int nsrc, int N, hipStream_t s);

void sx_launch_coef(const double *d, const int *base, int row0, int rows, double *coef, hipStream_t s);
void sx_launch_gemv_partials(const double *T, int rows, size_t ld, int Ns, const double *coef, double *partials,
                             hipStream_t s);
void sx_launch_gemv_apply(double *d, Cols c, const double *partials, int nblk, hipStream_t s);

void sx_launch_build_rows(double *T, int rows, int row0, size_t ld, int n, int m, int Ns, const double *A_local,
                          const double *b_full, hipStream_t s);
void sx_launch_init_vectors(double *d, int N1, int n, int m, int *base, hipStream_t s);
void sx_launch_phase2_costs(double *d, int n, int m, const double *c, hipStream_t s);
void sx_launch_gather_rhs(const double *T, int rows, size_t ld, double *out, hipStream_t s);
// device generator (sx_generator.hip) and the CRT seeding (sx_problem.cpp)
void sx_crt_seeds(unsigned seed, int kind, uint32_t out[3]);
void sx_launch_gen_rows(uint32_t seedA, int n, int m, int row0, int rows, double lo, double hi, double *T, size_t ld,
                        double *A_cm, hipStream_t s);
void sx_launch_gen_vector(uint32_t seed, long long first, int count, double lo, double hi, double *out,
                          hipStream_t s);

void sx_launch_argmin_vector(const double *v, long long L, TilePart *parts, int *out_idx, double *out_v,
                             hipStream_t s);
