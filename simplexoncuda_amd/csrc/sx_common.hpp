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
    int r;                 // leaving row (global) of the current pivot
    int pad0;
    double dmin;           // reduced cost of the entering variable (d[e+1] before the pivot)
    long long pivots;      // pivots selected in this phase
    long long max_pivots;  // < 0: no cap (reference behaviour)
    int e_next;            // entering argmin of the updated objective row (next pivot)
    unsigned ticket;       // arrival counter of the ratio/select hand-off (zero between launches)
    double dmin_next;      // its value
    unsigned ticket_d;     // arrival counter of the objective-row blocks of k_pivot_row
    unsigned batch_tag;    // batch id of the last selected pivot ...
    int batch_count;       // ... and the number of pivots selected in that batch
    int pad1;
};

// TilePart.elig: bit 0 = "some entry >= eps" of the tile (the unbounded test)
#define SX_ELIG(x) ((x) & 1)

// Deferred pivots: at most SX_KMAX pivots between two sweeps of the tableau.  A batch runs in
// stages of SX_HMAX slots (the on-chip history of the fused batch, the hand-off records, the
// per-pivot kernels, the vector sweep and the multi-rank batch hold one stage); the one-shard
// fused batch runs two stages, whose 64 pivots the matrix-core sweep applies at once.
#define SX_KMAX 64
#define SX_HMAX 32
// Position of row i's factor of slot s in F: rows in strips of 16, each strip slot-major
// ([strip][slot][16 rows]).  The matrix-core sweep's A operand for 4 slots of a 16-row strip is
// then 64 consecutive doubles (one coalesced load per 4-slot step), and a batch's per-pivot
// factor column is written 16 consecutive doubles per strip.  F holds round_up(rows, 16) rows.
__host__ __device__ constexpr size_t sx_fidx(long long i, int s) {
    return (size_t)(i >> 4) * (16 * SX_KMAX) + (size_t)s * 16 + (size_t)(i & 15);
}
// Batch ids run 1 .. SX_BATCH_IDS - 1: the fused kernels' granule tags keep 15 bits of the id
// (sx_kernels.hip make_tag).  When the ids wrap, the engine clears every id-tagged word (the
// PM pending-leaving masks and the granule records) first, so no stale tag can match.
#define SX_BATCH_IDS (1u << 15)

// Record of one pending pivot (slot s of the current batch).
struct __attribute__((aligned(16))) PivRec {
    int r;     // leaving row (global)
    int e;     // entering variable
    double p;  // pivot element
};

// Device buffers of the pending pivots of a shard, plus the batch id and slot of the pivot
// being enqueued (kernel arguments).
struct Pending {
    // [SX_KMAX][ld] pivot rows (current leaving-row values, before /p).  INVARIANT every writer keeps
    // (k_pivot_row, k_batch / k_batch_mr objective tiles, k_select_row / the row gathers' remote
    // rows, k_activate / activate_block's column exchanges): U[s][j] is the EXACT current value of
    // row r_s at stored column j < Ns just before slot s -- the reference's bits -- for every stored
    // column the sweep touches.  The sweep's leaving-row fix-up (msweep_fixup) and the ratio tiles'
    // leaving-row shortcut restart a row that left at slot sl from U[sl][j] / p_sl instead of its
    // stored value, so they are correct only under this invariant
    // (tests/test_gpu_parity.py::test_row_leaves_twice_per_stage_compacted).
    double *U;
    double *F;               // row factors -(a_ie / p), F[sx_fidx(i, s)]
    PivRec *recs;            // [SX_KMAX]
    unsigned long long *PM;  // [rows] (batch id << 32) | slots < SX_HMAX where the row left the basis
    unsigned long long *PM2; // [rows] the same for slots SX_HMAX + b (bit b): the second stage
    unsigned batch;          // id of the current batch (never 0)
    int q;                   // slot of the pivot being enqueued (pivots pending before it)
};

// Fused batch kernel (k_batch): its exit counter and abort word, each on its own line.
// (The per-pivot hand-offs are data-tagged granules in two arrays of tile records,
// sx_batch_granules_a/b() 8-byte words each.)
struct BatchChan {
    alignas(128) unsigned exit_cnt;  // blocks that have left the kernel
    alignas(128) unsigned abort_w;   // a wait timed out: every block leaves
    alignas(128) unsigned inject_q;  // test hook: 1 + the slot at which ratio block 0 (of rank 0)
                                     // leaves with the batch aborted (0: off); the last block clears it
};

// Multi-rank fused batch (k_batch_mr): every rank's buffers as seen from this rank (peer
// memory over xGMI, or the other virtual shards on one GPU).
#define SX_MAXW 8
struct PeerView {
    const double *T[SX_MAXW];        // tableaux (read: the leaving row)
    unsigned long long *ga[SX_MAXW]; // ratio-tile records (written)
    unsigned long long *gb[SX_MAXW]; // objective-tile records (written)
    unsigned long long *gdone[SX_MAXW];  // batch-end done granules (written)
    double *U[SX_MAXW];              // pending pivot rows (written)
    const double *F[SX_MAXW];        // pending row factors (read: the leaving row's first stage)
    double *d[SX_MAXW];              // objective rows (written)
};

#define SX_HANG (-13)  // fused batch kernel: a hand-off wait timed out (never expected; the host
                       // restores the batch's start state and re-runs it on the per-pivot path)

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
//
// Slack compaction: while row k has never been a leaving row, its slack
// column is exactly e_k and every pivot leaves it bit-identical (its pivot-row entry is +0).
// Such columns are kept at the end of the stored slack block and the sweep stops before
// them: stored slack position s0 + perm[k] holds logical slack k, and the first *nact
// positions are the columns that have ever been touched.
struct Cols {
    int N;      // logical columns of the phase (reference width: 1+n+2m or 1+n+m)
    int Ns;     // stored columns
    int art0;   // first aliased logical column, or INT_MAX
    int shift;  // alias distance (m)
    int s0;     // first slack column (1+n)
    const int *perm;  // device: logical slack -> stored slack offset, or null (identity)
    __host__ __device__ __forceinline__ int map(int j) const {
        const int k = j >= art0 ? j - shift : j;
        return (perm && k >= s0) ? s0 + perm[k - s0] : k;
    }
};

// Tableau storage in HBM: two regions.  Region A holds stored columns [0, jB) of
// every row at stride ldA; region B, starting offB doubles later, holds stored columns [jB, Ns)
// at stride ldB.  With slack compaction the swept columns [0, 1 + n + nact) lie in region A while
// nact fits, so the sweep streams dense rows (a row of A is only a little wider than what is
// swept) instead of a prefix of every full-width row; without a region B (jB = Ns, the default for
// small m and for callers' tableaux) there is one region.  jB is a multiple of 512, so no
// 512-column tile straddles the two.
// Inside a region, blk = 0: plain row-major (callers' tableaux: tabular.h); blk = 1 (the engine's
// own tableaux): 16-row strips of ld * 16 doubles, each strip a sequence of 4-column
// groups of 64 doubles, each group 4 blocks of 4 rows x 4 columns (one 128-byte line each).  A
// column of 512 rows then spans 128 lines instead of 512 (the fused batch's entering-column
// gather), a row's 512 columns 128 lines instead of 32 (its pivot-row read), and a strip is still
// one contiguous range (the sweep); two adjacent columns 2c, 2c + 1 of a row stay adjacent.
// Rows are allocated in whole strips.
struct TLay {
    size_t ldA = 0, ldB = 0, offB = 0;
    int jB = 0x7fffffff;
    int blk = 0;
    __host__ __device__ __forceinline__ static size_t b4(long long i, int j, size_t ld) {
        return (size_t)(i >> 4) * 16 * ld + (size_t)(j >> 2) * 64 + (size_t)(((int)i & 15) >> 2) * 16 +
               (size_t)(((int)i & 3) * 4 + (j & 3));
    }
    __host__ __device__ __forceinline__ size_t idx(long long i, int j) const {
        if (blk) return j < jB ? b4(i, j, ldA) : offB + b4(i, j - jB, ldB);
        return j < jB ? (size_t)i * ldA + (size_t)j : offB + (size_t)i * ldB + (size_t)(j - jB);
    }
};

// ---- kernel launchers (sx_kernels.hip) ----
struct SweepCfg {
    int batch;  // pivots per sweep (1..SX_KMAX; the vector sweep: up to SX_HMAX)
    int mfma;   // 1: the matrix-core sweep (k_msweep), 0: the vector sweep (k_sweep)
};

int sx_enter_blocks(int L);
void sx_launch_enter(const double *d, int L, TilePart *parts, DevState *st, hipStream_t s);
void sx_launch_ratio_select(const double *T, int rows, int row0, size_t ld, TLay tl, TilePart *tiles_local, double *colE,
                            DevState *st, int *base, bool select, double *slots, size_t slot_stride, Cols c,
                            const Pending &pd, hipStream_t s);
void sx_launch_select_gathered(const double *slots, size_t slot_stride, int B2, int *base, DevState *st,
                               const Pending &pd, hipStream_t s);
void sx_launch_select_row(const double *T, int rows, int row0, size_t ld, TLay tl, Cols c, const TilePart *tiles_all, int B2,
                          double *prow_out, int *base, DevState *st, const Pending &pd, hipStream_t s);
void sx_launch_pivot_row(const double *T, int rows, int row0, size_t ld, TLay tl, Cols c, double *d, const double *prow_buf,
                         size_t prow_stride, const double *colE, DevState *st, const Pending &pd,
                         TilePart *enter_parts, hipStream_t s);
// nact (device, or null): sweep only the columns [0, s0 + *nact) (slack compaction)
void sx_launch_sweep(double *T, int rows, int row0, size_t ld, TLay tl, int Ns, const int *nact, int s0,
                     const Pending &pd, const DevState *st, int rev, SweepCfg cfg, hipStream_t s);
// slack compaction, after a batch's selections and before its sweep: move the slack column
// of every row that left the basis for the first time into the swept block
// (ucol[r]: the unswept slack column that is the unit vector e_r, or -1; urow[k]: the row of unswept
// slack k's unit vector -- k itself until row k first leaves)
void sx_launch_activate(int *perm, int *iperm, int *ucol, const int *urow, int *nact, int m, double *T, int rows,
                        int row0, size_t ld, TLay tl, int s0, const Pending &pd, const DevState *st, int slots,
                        hipStream_t s);  // slots: the batch size (two passes above SX_HMAX)
// one shard, after a sweep (every few batches): the swept slack columns whose slack is basic (exact
// unit vectors, checked) moved behind the swept block (k_deact_*)
#define SX_DEACT_CAP 4096  // columns per round (a multiple of 1024)
struct DeactList {
    int C;    // listed columns (swept slacks that are basic), stored-position order
    int nsw;  // column exchanges of the round
    int x[SX_DEACT_CAP], r[SX_DEACT_CAP], bad[SX_DEACT_CAP];  // position, unit row, failed the check
    int dst[SX_DEACT_CAP], src[SX_DEACT_CAP], row[SX_DEACT_CAP];
};
// (tag: [m] position tags, zero at allocation; epoch: this round's number, from 1; check: compare each
// column with its unit vector first -- required: an entered column is e_r only where its entries'
// residuals a_k - fl(a_k / p) p round to 0; fail: [m] slack -> 1 + the row it failed the check in, zero
// at allocation)
void sx_launch_deactivate(int *perm, int *iperm, int *ucol, int *urow, int *nact, const int *base, int n, int m,
                          bool alias, double *T, int rows, int row0, TLay tl, int s0, unsigned long long *tag,
                          unsigned epoch, bool check, int *fail, DeactList *L, hipStream_t s);
// fused batch of up to k pivots on one shard (ratio tiles + objective tiles in one resident
// grid); returns false (nothing launched) when the grid cannot be resident at once
bool sx_batch_fits(int rows, Cols c, int k);
int sx_batch_obj_tile_limit();  // objective tiles a one-shard fused batch holds (logical width <= 512 x this + 1)
// d_save: the objective row as the batch found it (restored by the host after SX_HANG); the
// basis is written only by a batch that completed
// perm / iperm / ucol / urow / nact (slack compaction, or null): the batch's last block also activates
// the slack columns of the rows that left the basis for the first time (k_activate's work)
void sx_launch_batch(const double *T, int rows, size_t ld, TLay tl, Cols c, double *d, double *d_save, int *base,
                     DevState *st, const Pending &pd, int k, BatchChan *chan, unsigned long long *ga,
                     unsigned long long *gb, unsigned long long *stamps, int *perm, int *iperm, int *ucol,
                     const int *urow, int *nact, int m, hipStream_t s);
size_t sx_batch_granules_a();
size_t sx_batch_granules_b();
// the multi-rank fused batch: `grids` co-resident launches of this shape must fit the device
bool sx_batch_mr_fits(int slots, int nb_local, int k, int grids);
void sx_launch_batch_mr(const double *T, int rows, int row0, int rpr, size_t ld, TLay tl, Cols c, double *d, double *d_save,
                        int *base, DevState *st, const Pending &pd, int k, int slots, int W, int rank, int tb0, int tb1,
                        int repl, BatchChan *chan, const unsigned long long *ga, const unsigned long long *gb,
                        const unsigned long long *gdone, const PeerView &pv, unsigned long long timeout,
                        hipStream_t s);
// one rank of a multi-rank launch
struct MrLaunchRank {
    const double *T;
    int rows, row0, rank, tb0, tb1;
    int repl;  // replicated objective: every rank runs every objective tile (tb0 = 0, tb1 = all)
    const int *perm;
    double *d, *d_save;
    int *base;
    DevState *st;
    Pending pd;
    BatchChan *chan;
    const unsigned long long *ga, *gb, *gdone;
};
// the batches of the nloc ranks (of W) that share one GPU, as one launch
void sx_launch_batch_mr_multi(const MrLaunchRank *ranks, int nloc, int W, int rpr, size_t ld, TLay tl, Cols c, unsigned B,
                              int k, int slots, const PeerView &pv, unsigned long long timeout, hipStream_t s);
void sx_set_update_waves(float w);  // resident-grid multiple of the sweep (default 1)
void sx_set_sweep_record(int *rec);  // next sweeps write (batch tag, count, nact) to rec[0..2] (null: off)
void sx_launch_sum_rows(double *out, const double *const *srcs, int nsrc, int N, hipStream_t s);
void sx_launch_l2_writeback(hipStream_t s);  // every XCD's L2 writes back its dirty lines
// diagnostic: every shard's pending pivot rows of batch B against shard 0's (counts mismatches in *bad)
void sx_launch_check_u(const PeerView &pv, int W, size_t ld, int Ns, const DevState *st, unsigned B,
                       unsigned long long *bad, hipStream_t s);
// a rank's contribution to the objective-row gather: d on [j0, j1) (and d[0] if with0), -0.0 elsewhere
void sx_launch_d_contrib(const double *d, double *out, int N, int j0, int j1, int with0, hipStream_t s);

void sx_launch_coef(const double *d, const int *base, int row0, int rows, double *coef, hipStream_t s);
void sx_launch_gemv_partials(const double *T, int rows, TLay tl, int Ns, const double *coef, double *partials,
                             hipStream_t s);
void sx_launch_gemv_apply(double *d, Cols c, const double *partials, int nblk, hipStream_t s);

void sx_launch_build_rows(double *T, int rows, int row0, TLay tl, int n, int m, int Ns, const double *A_local,
                          const double *b_full, hipStream_t s);
void sx_launch_init_vectors(double *d, int N1, int n, int m, int *base, hipStream_t s);
void sx_launch_phase2_costs(double *d, int n, int m, const double *c, hipStream_t s);
void sx_launch_gather_rhs(const double *T, int rows, TLay tl, double *out, hipStream_t s);
// rows [i0, i0 + nr), stored columns [0, Ns) -> row-major out (nr x Ns); and row-major in (pitch
// ld_in) -> stored columns [j0, j0 + Ns) of those rows
void sx_launch_rows_out(const double *T, TLay tl, int i0, int nr, int Ns, double *out, hipStream_t s);
void sx_launch_rows_in(double *T, TLay tl, int i0, int nr, int Ns, int j0, const double *in, size_t ld_in,
                       hipStream_t s);
// device generator (sx_generator.hip) and the CRT seeding (sx_problem.cpp)
void sx_crt_seeds(unsigned seed, int kind, uint32_t out[3]);
void sx_launch_gen_rows(uint32_t seedA, int n, int m, int row0, int rows, double lo, double hi, double *T, TLay tl,
                        double *A_cm, hipStream_t s);
void sx_launch_gen_vector(uint32_t seed, long long first, int count, double lo, double hi, double *out,
                          hipStream_t s);

void sx_launch_argmin_vector(const double *v, long long L, TilePart *parts, int *out_idx, double *out_v,
                             hipStream_t s);
