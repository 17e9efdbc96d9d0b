/*
 * simplex_hip.h -- MI355X engine extensions of the C-ABI (libsimplex_hip.so).
 *
 * Nothing here exists in the reference; it is what a benchmark, a parity test or a
 * multi-GPU launcher needs on top of the drop-in entry points (twoPhaseMethod.h).
 * Plain C types only.
 */
#ifndef SIMPLEX_HIP_H
#define SIMPLEX_HIP_H

#include "problem.h"
#include "tabular.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SIMPLEX_NOT_ENDED -10    /* solver.cu:77 */
#define SIMPLEX_PIVOT_CAP -11    /* opt-in pivot budget reached */
#define SIMPLEX_NUMERIC_FAIL -12 /* eligible pivot but the ratio argmin found no row */
#define SIMPLEX_HANG -13         /* fused batch: an in-kernel hand-off timed out (never expected) */
#define SIMPLEX_MAX_GPUS 8        /* shards (GPUs) one solve can use: simplex_set_gpus, SIMPLEX_GPUS, --gpus */

/* ---- configuration ---- */
int simplex_version(void);
void simplex_set_verbose(int on);            /* reference progress lines on stdout */
/* the sweep on the matrix cores (v_mfma_f64_16x16x4f64, bit-identical to the vector chain):
 * -1 auto (matrix cores), 0 vector sweep (batches of at most 32), 1 matrix-core sweep */
void simplex_set_sweep_mfma(int mode);
/* pivots per tableau sweep (1..64; 0 = auto: 64 when the tableau has >= 4096 rows -- two stages
 * of 32, applied by the matrix-core sweep -- else 32; more than 32 only in the fused batches, one
 * shard's and the peer-memory multi-rank one, the per-pivot path caps it at 32): the pivots of a
 * batch are selected on the
 * current values (pending pivots applied on the fly) and then applied to the tableau in one
 * sweep -- the same IEEE operations in the same order as one sweep per pivot */
void simplex_set_batch(int pivots);
void simplex_set_device(int device);
/* write the reference's -D TIMER CSV (chrono.cu) into `dir` (NULL or "" = off; env
 * SIMPLEX_TIMER_DIR also enables it); benchmark mode names it benchmark_<n>_<m>.txt */
void simplex_set_timer_dir(const char *dir);

/* ---- multi-GPU: one process per GPU, RCCL communicator over xGMI ---- */
int simplex_dist_unique_id_size(void);
int simplex_dist_get_unique_id(unsigned char *out); /* rank 0; out has unique_id_size bytes */
int simplex_dist_init(int rank, int world, const unsigned char *unique_id, int device);
int simplex_dist_finalize(void);
/* single-process emulation of W row-block shards on the current device (collectives are
 * device copies); used to test the sharded path on one GPU. 0 or 1 disables. */
void simplex_set_virtual_ranks(int world);
/* ---- multi-GPU inside ONE process: the caller still makes one synchronous
 * twoPhaseMethod / solve call.  The constraint rows are split into count 512-aligned blocks, one
 * per listed device (a device may repeat); the shards hand off through peer memory (one fused
 * launch per device per batch of pivots) when a start-up self-check on the list passes, else
 * through per-pivot device copies.  Without this call the environment variable SIMPLEX_GPUS
 * decides: "N" = devices 0..N-1, or a comma list ("0,1,2,3").  count <= 1 (or no list): one
 * shard.  A device that is not visible is a fatal error (error.cu:5-12 convention). */
void simplex_set_gpus(const int *devices, int count);
/* the device list in effect (simplex_set_gpus, else SIMPLEX_GPUS); returns its length and
 * copies up to cap entries */
int simplex_gpus(int *devices, int cap);
/* run the multi-shard exchange path (tile allgather + pivot-row allreduce) even with a
 * single shard; with simplex_dist_init(.., world=1, ..) it goes through a 1-rank RCCL
 * communicator.  Test hook. */
void simplex_set_force_exchange(int on);
/* per-pivot exchange between shards: 0 auto, 1 tile-winner allgather + pivot-row allreduce,
 * 2 one allgather of tile winners together with their rows (auto: when <= 1 MiB per rank) */
void simplex_set_exchange_mode(int mode);
/* store each phase-1 artificial column as its (bit-identical) slack column: 1 on (default), 0 off */
void simplex_set_alias(int on);
/* slack compaction (default on): the slack column of a row that has never left the basis is
 * an untouched unit vector, so it is kept past the swept block of the tableau and skipped by
 * every sweep -- bit-identical results; active only when no row is negated (b >= 0) */
void simplex_set_compact(int on);
/* with slack compaction on one shard: every `every` sweeps (default 8; 0 off) the swept slack
 * columns whose slack is basic -- exact unit vectors, checked bit for bit -- are moved past the swept
 * block too, and moved back when their row leaves; bit-identical results */
void simplex_set_deactivate(int every);
/* one shard: run each batch of pivots as ONE resident launch (ratio tiles + objective-row tiles
 * handing off through write-through records) instead of two launches per pivot;
 * -1 auto (default: when the grid fits the device), 0 off */
void simplex_set_fused(int mode);
/* several shards: run each batch as ONE launch per rank whose ranks hand off through peer
 * memory (xGMI; virtual shards: the same device) instead of per-pivot RCCL calls; -1 auto
 * (default: RCCL ranks when the start-up self-check in simplex_dist_init passed), 0 off,
 * 1 force (virtual shards: only with 1; all ranks' batches as one launch, or with
 * simplex_set_mr_single_launch(0) one launch per rank for W <= 3) */
void simplex_set_p2p(int mode);
/* 1 when the peer-memory fused path passed simplex_dist_init's self-check on every rank */
int simplex_p2p_ready(void);
/* how the shards of this process (RCCL ranks, or the SIMPLEX_GPUS device list) passed their
 * start-up self-check against a one-shard solve of the same instance: 2 peer-memory fused batches,
 * 1 the per-pivot exchange, 0 neither (every solve then runs on one device: RCCL ranks each solve
 * alone, a device list on its first device), -1 not checked (yet) or one shard */
int simplex_multi_gpu_mode(void);
/* wall time (s) of the last twoPhaseMethod call's two pivot loops (solve calls): out[0] phase 1,
 * out[1] phase 2 -- the reference's TIMER CSV reports the two phases separately */
void simplex_last_phase_seconds(double *out);
/* the last twoPhaseMethod call's final objective row d[0, N) in logical columns (N = 1+n+m after
 * phase 2, 1+n+2m when phase 1 ended the solve): copies min(N, cap) entries, returns N.  After a
 * FEASIBLE solve, d[1+n+i] = y_i (the dual of constraint i, also for the rows negated by the b < 0
 * quirk, twoPhaseMethod.cu:100-111) and d[1+j] = (A^T y)_j - c_j: a dual certificate */
long long simplex_last_objective_row(double *out, long long cap);
/* the sweep's grid: waves x (blocks resident on the device) blocks (default 1; <= 0 resets) */
void simplex_set_update_waves(double waves);
/* new engines' tableau layout: plain row-major rows (0), the two-region layout when aliasing and
 * m > 4096 (1, default), or region A forced to hold `mode` slack positions (>= 2,
 * test hook) */
void simplex_set_regions(int mode);
/* virtual shards with the peer-memory batch: every rank's batch in one launch (1, default) or one
 * launch per rank on its own stream (0; needs as many hardware queues running at once) */
void simplex_set_mr_single_launch(int on);

/* the pending pivot rows U (written by peer ranks in the multi-rank batch) in fine-grained memory:
 * -1 auto (when the shards span devices, default), 1 always (test hook: the one-GPU cost and
 * parity of that path), 0 never; 2 (test hook): uncached memory for exchanging shards, the
 * allocation of the round-4/5 divergence */
void simplex_set_fine_pivot_rows(int mode);
/* multi-rank fused batches with the objective row replicated: every rank runs every objective
 * tile (decides the entering variable and forms the whole pivot row itself), so a pivot's only
 * cross-rank hand-offs are the ratio tiles' winners and the leaving row read from its owner
 * (DESIGN.md §5.2): -1 auto (when the shards span devices, default), 1 always (when the grid of
 * slots + every objective tile per rank fits; else the split objective), 0 never (each rank runs
 * its share of the objective tiles and the records go to every rank) */
void simplex_set_replicated_objective(int mode);
/* new engines' tableau storage inside each region: -1 default (blocks of 4 rows x 4 columns in
 * 16-row strips, unless the environment sets SIMPLEX_BLOCKED=0), 1 blocked, 0 plain row-major
 * (callers' tableaux, tabular.h, are always row-major) */
void simplex_set_blocked(int mode);

/* ---- fault handling and test hooks ---- */
/* a fused batch whose in-kernel hand-off wait times out (SIMPLEX_HANG, never expected) is
 * undone and re-run on the per-pivot path; this counts such recoveries in the process */
long long simplex_hang_recoveries(void);
long long simplex_fused_batches(void);           /* fused batch launches in the process */
/* diagnostic: before every sweep of a multi-shard engine of this process (virtual shards, a
 * SIMPLEX_GPUS list), compare every shard's pending pivot rows U with shard 0's bit for bit and
 * count (and print the first) mismatches -- 1 on, 0 off (default; SIMPLEX_CHECK_PIVOT_ROWS=1 also
 * turns it on).  Synchronous per batch: for tests and diagnosis, not for timing */
void simplex_set_check_pivot_rows(int on);
long long simplex_pivot_row_mismatches(void);    /* mismatches counted in the process */
/* test hook: make the n-th fused batch from now abort as if a wait had timed out (-1 off) */
void simplex_set_hang_inject(long long batches);
/* ... at which slot of that batch: -1 (default) before it starts; s >= 0: the batch runs s
 * pivots (the objective row already updated by them) and then one block leaves it, so the others
 * time out inside the batch */
void simplex_set_hang_inject_slot(int slot);
/* test hook: batch id of the next engine's first batch (1 .. 32767; ids wrap at 32768) */
void simplex_set_first_batch_id(unsigned int id);

/* ---- extended drop-in entry ---- */
/* twoPhaseMethod + final basis (base_out[m]) and per-phase pivot counts (pivots_out[2]);
 * max_pivots < 0 = no cap (parity mode), else per-phase cap (status SIMPLEX_PIVOT_CAP).
 * It returns the engine-only statuses (SIMPLEX_PIVOT_CAP, SIMPLEX_NUMERIC_FAIL, SIMPLEX_HANG)
 * as such; twoPhaseMethod and solve keep the reference contract (0/-1/-2/-3, solve 0/-2) and
 * treat NUMERIC_FAIL and HANG as fatal errors (print, exit; error.cu:5-12). */
int twoPhaseMethodEx(problem_t *problem, double *solution, double *optimalValue, int *base_out,
                     long long *pivots_out, long long max_pivots);

/* problem_t from caller arrays (copied; A column-major m x n); free with freeProblem()
 * and then free() of the struct, as the reference's callers do. */
problem_t *simplex_problem_from_arrays(int n, int m, const double *A_colmajor, const double *b,
                                       const double *c);
/* the generator with an explicit CRT flavour: 0 = MSVC rand() (default, matches the
 * published pivot counts), 1 = glibc rand() */
problem_t *simplex_generate_problem_ex(int n, int m, unsigned int seed, int lo, int hi, int rand_kind);
void simplex_free_problem_struct(problem_t *problem);
/* generateRandomProblem computed on the GPU (jump-ahead XORWOW, one thread per row chunk, as
 * the reference's generator.cu does on its GPU); bit-identical to the host generator */
problem_t *simplex_generate_problem_device(int n, int m, unsigned int seed, int lo, int hi, int rand_kind);

/* ---- benchmark session: a resident phase-1 tableau and timed pivots ---- */
typedef struct {
    double wall_ms;            /* device time of the whole call (events on the engine stream) */
    double update_ms;          /* sum of the timed sweep kernel durations (HIP events) */
    long long pivots;          /* pivots applied during the call */
    long long update_launches; /* sweeps timed (those that applied at least one pivot) */
    int status;                /* phase status after the call (SIMPLEX_NOT_ENDED while running) */
    int width;                 /* tableau width N of the phase (reference counting) */
    int stored_width;          /* columns stored (artificials alias slacks in phase 1); a sweep moves all
                                * of them, or 1+n+(touched slacks) under slack compaction */
    long long local_rows;      /* constraint rows owned by this process */
    double update_bytes;       /* bytes per sweep: 16 * local_rows * swept width (read + write of T),
                                * the mean over the timed sweeps */
    long long swept_pivots;    /* timed sweeps: pivots they applied */
    double swept_bytes;        /* timed sweeps: bytes they moved */
} simplex_timing_t;

typedef struct simplex_session simplex_session;
simplex_session *simplex_session_open(problem_t *problem); /* builds phase 1 + canonicalises d */
/* same tableau as simplex_session_open(generateRandomProblem(n, m, seed, lo, hi)), synthesised
 * directly in HBM (each shard generates only its rows; no host copy of A) */
simplex_session *simplex_session_open_generated(int n, int m, unsigned int seed, int lo, int hi, int rand_kind);
/* k pivots (the call ends with a sweep, so the tableau is materialised on return);
 * time_updates = s > 0 brackets every s-th sweep with HIP events */
int simplex_session_pivots(simplex_session *s, long long k, int time_updates, simplex_timing_t *out);
double simplex_session_objective(simplex_session *s);   /* d[0] */
/* the resident tableau in logical column order (m rows of the phase's width at stride ld; T
 * null: not copied), the objective row d and the basis; returns the width, or -1 when rows live
 * on other ranks or the buffer is too narrow */
long long simplex_session_tableau(simplex_session *s, double *T, long long ld, double *d, int *base);
/* slack columns the sweeps currently move (m without slack compaction) */
long long simplex_session_active_slacks(simplex_session *s);
long long simplex_session_total_pivots(simplex_session *s);
/* pivots per batch (and per sweep) of simplex_session_pivots on this session */
int simplex_session_batch(simplex_session *s);
/* per timed sweep of the last simplex_session_pivots call: pivots it applied and its
 * duration in microseconds; returns the number of sweeps logged (at most cap are copied) */
long long simplex_session_launch_log(simplex_session *s, long long *rows, double *update_us, long long cap);
/* diagnostic: one fused batch of k pivots with in-kernel timestamps (100 MHz ticks) at the
 * hand-off points, out[k][8]: 0 ratio block 0 starts the pivot, 2 its ratios computed, 1 its
 * tile published, 3 objective block 0 knows the selection, 6 it has the leaving row's details,
 * 7 its pivot-row values, 4 its tile published, 5 ratio block 0 knows the next entering
 * variable; -1 when the fused path is not in use */
int simplex_session_stamps(simplex_session *s, int k, unsigned long long *out);
/* the same with every block's own stamps, blk[k][blocks][4] (ratio blocks first: starts the pivot,
 * tile published, knows the next entering variable; objective blocks: knows the selection, has
 * the details, tile published), copied when cap >= k * blocks * 4; returns the blocks (-1 as above) */
int simplex_session_block_stamps(simplex_session *s, int k, unsigned long long *out, unsigned long long *blk,
                                 long long cap);
void simplex_session_close(simplex_session *s);

/* ---- multi-process peer-memory test mode (no RCCL; e.g. 2 processes on one GPU) ----
 * Each process owns rank `rank` of `world` row-block shards (512-aligned blocks, as
 * simplex_dist_init would make them) of a phase-1 state given in logical columns: T_rows =
 * this rank's rows (ld_host doubles apart, width 1+n+2m), d and base whole.  The session's
 * six peer-visible buffers are exported as IPC handles (simplex_ipc_handles_size() bytes);
 * the caller gathers every rank's handles (rank order) and connects; simplex_session_pivots
 * then runs fused multi-rank batches whose hand-offs cross the processes through those
 * mappings.  Returns NULL / < 0 on failure.  Keep every process alive until all have
 * finished their pivots before closing. */
int simplex_ipc_handles_size(void);
simplex_session *simplex_ipc_session_open(int n, int m, int rank, int world, const double *T_rows, long long ld_host,
                                          const double *d, const int *base, unsigned char *handles_out);
int simplex_ipc_session_connect(simplex_session *s, const unsigned char *all_handles);
/* after every process's pivots: write this rank's slice of the objective row into every peer's
 * (between fused batches each rank keeps only its own slice current); barrier the processes
 * before and after.  Returns 0, or -1 for a session that is not in IPC mode. */
int simplex_session_sync_d(simplex_session *s);
/* this process's rows of the resident tableau (logical columns), d and base; returns rows, -1 for
 * ld_host < N, -2 for an IPC session whose objective row is split after its pivots (call
 * simplex_session_sync_d in every process first) */
long long simplex_session_rows(simplex_session *s, double *T_rows, long long ld_host, double *d, int *base);

/* ---- kernel bench (SURVEY.md §8d config 3') ---- */
/* the sweep kernel (solver.cu:34-46's update, `pivots` pending pivots per pass) on a synthetic
 * rows x cols fp64 matrix drawn like generateRandomProblem's A (seed, values in [lo, hi]) with
 * random pending pivots; `warmup` untimed then `iters` timed sweeps (HIP events); returns the
 * average microseconds per sweep (< 0 on bad arguments), *bytes = 16 * rows * cols */
double simplex_bench_sweep(int rows, int cols, unsigned int seed, int lo, int hi, int pivots, int warmup, int iters,
                           double *bytes);

/* ---- kernel-level parity hooks (host arrays in/out, device compute) ---- */
/* epsilon argmin of v[0..L) with the reference combine tree; returns index (or -1) */
long long simplex_dev_argmin(const double *v, long long L, double *vmin);
/* k full pivots on a caller tableau (row-major m x ld, width N) + d + base; returns the
 * phase status after them (SIMPLEX_NOT_ENDED if still running); *done = pivots applied */
int simplex_dev_pivots(double *T, long long m, long long N, long long ld, double *d, int *base, long long k,
                       long long *done);
/* objective canonicalisation d[j] -= sum_i T[i][j] * d[1+base[i]] on the device */
int simplex_dev_update_objective(const double *T, long long m, long long N, long long ld, const int *base,
                                 double *d);
/* phase-1 tableau as built on the device (row-major m x ld, ld >= 1+n+2m), d and base */
int simplex_dev_build_phase1(problem_t *problem, double *T, long long ld, double *d, int *base);
/* the same from the device generator */
int simplex_dev_build_phase1_generated(int n, int m, unsigned int seed, int lo, int hi, double *T, long long ld,
                                       double *d, int *base);

#ifdef __cplusplus
}
#endif
#endif
