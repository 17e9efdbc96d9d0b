// sx_engine.cpp -- host side of the MI355X simplex: shards, the device-resident pivot
// loop, the two-phase driver and the C-ABI entry points of include/*.h.
//
// Reference call structure replaced: twoPhaseMethod (twoPhaseMethod.cu:385)
// -> phase1/phase2 (:225, :285) -> solve (solver.cu:128) -> per-iteration solve (:78).
// The reference crosses PCIe ~10 times per pivot (blocking copies, mallocs, syncs).  Here a
// pivot is two kernels (plus, on several GPUs, one or two RCCL collectives) enqueued on one
// stream, and the tableau itself is swept once per batch of pivots (deferred rank-1 updates,
// DESIGN.md §3); the host only polls a pinned status word once per batch.
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <ctime>
#include <functional>
#include <map>
#include <string>
#include <mutex>
#include <vector>

#include "../../include/simplex_hip.h"
#include "../../include/twoPhaseMethod.h"
#include "sx_common.hpp"
static_assert(SX_MAXW == SIMPLEX_MAX_GPUS, "simplex_hip.h SIMPLEX_MAX_GPUS is the engine's shard limit");

// ------------------------------------------------------------------ errors (error.cu:5-18)
void sx_handle_error(hipError_t err, const char *file, int line) {
    if (err != hipSuccess) {
        printf("%s in %s at line %d\n", hipGetErrorString(err), file, line);
        fflush(stdout);
        exit(EXIT_FAILURE);
    }
}

void sx_fatal(const char *msg, const char *file, int line) {
    printf("%s in %s at line %d\n", msg, file, line);
    fflush(stdout);
    exit(EXIT_FAILURE);
}

static void nccl_check(ncclResult_t r, const char *file, int line) {
    if (r != ncclSuccess) {
        printf("%s in %s at line %d\n", ncclGetErrorString(r), file, line);
        fflush(stdout);
        exit(EXIT_FAILURE);
    }
}
#define SX_NCCL(call) nccl_check((call), __FILE__, __LINE__)

// ------------------------------------------------------------------ global configuration
namespace {

struct Config {
    int verbose = 0;
    int sweep_mfma = -1;  // the matrix-core sweep: -1 auto, 0 off, 1 on
    int batch = 0;           // pivots per tableau sweep (deferred updates), 1..SX_KMAX; 0 = auto
    int device = -1;
    int virtual_ranks = 1;
    std::vector<int> gpus;   // simplex_set_gpus: one process, one row-block shard per listed device
    int force_exchange = 0;  // run the multi-shard exchange path even with one shard
    std::string timer_dir;   // non-empty: write the reference's TIMER CSV there
    int exchange_mode = 0;   // 0 auto, 1 tile allgather + row allreduce, 2 row-gather
    int alias = 1;           // store phase-1 artificial columns as their slack columns
    int compact = 1;         // sweep only the slack columns pivots have touched (when exact)
    int deact = -1;          // ... and move the swept slacks that are basic out of the sweep every `deact`
                             // sweeps (one shard; 0 off; -1: SIMPLEX_DEACTIVATE=k, else 8)
    int mr_single_launch = 1;  // virtual shards: all ranks' fused batches as one launch (0: one per stream)
    int regions = 1;         // two-region tableau layout (TLay): 0 off, 1 auto (aliasing, m > 4096),
                             // >= 2: region A holds that many slack positions (test hook)
    int fused = -1;          // whole batches in one resident launch: -1 auto (one shard), 0 off
    int p2p = -1;            // several shards: fused batches exchanging over peer memory: -1 auto, 0 off, 1 force
    bool p2p_ready = false;  // RCCL ranks: the peer-memory path passed the start-up self-check
    std::map<std::vector<int>, int> gpus_checked;  // one process, several GPUs: self-check result per device list
    // ... of a check run with peer memory off (simplex_set_p2p(0): only the per-pivot exchange checked, so
    // its result says nothing about the peer-memory batches and is not reused once they are enabled)
    std::map<std::vector<int>, int> gpus_checked_xchg;
    // diagnostic (simplex_set_check_pivot_rows / SIMPLEX_CHECK_PIVOT_ROWS=1): before every sweep of
    // a multi-shard engine of this process, every shard's pending pivot rows against shard 0's
    int check_u = -1;
    long long u_mismatches = 0;
    bool single_shard = false;  // every engine one shard on its own device (self-check reference; the
                                // fallback when the shards' exchange failed the self-check)
    int debug = -1;          // -1: from SIMPLEX_DEBUG; 1: print the tableau after every step
    bool benchmark = false;
    bool no_timer = false;         // the multi-GPU self-check: never write TIMER CSVs
    long long inject_hang = -1;    // test hook: abort the n-th fused batch from now (-1 off)
    int inject_slot = -1;          // ... before it starts (-1) or at this slot (inside the kernel)
    int mr_two_stage = -1;         // peer-memory multi-rank batches of two stages (-1: unless SIMPLEX_MR_STAGES=1)
    unsigned first_batch_id = 1;   // test hook: batch id of a new engine's first batch
    int fine_u = -1;               // U in fine-grained memory: -1 across devices, 1 always, 0 never
    int repl_obj = -1;             // replicated objective in multi-rank batches: -1 across devices, 1 always, 0 never
    int blocked = -1;              // the engine's tableaux in 4x4 blocks (TLay::blk): -1 default (off unless
                                   // SIMPLEX_BLOCKED=1), 0 row-major, 1 blocked
    int ipc_rank = -1, ipc_world = 0;  // test hook: one shard per process, peers through IPC handles, no RCCL
    long long hang_recoveries = 0; // fused batches aborted and re-run on the per-pivot path
    long long fused_batches = 0;   // fused batch launches (every shard's counted once)
    // distributed
    bool dist = false;
    int rank = 0;
    int world = 1;
    ncclComm_t comm = nullptr;
};

Config g_cfg;
std::mutex g_mu;

// The granule records of the RCCL ranks' peer-memory batch are polled inside a launch while
// other GPUs write them, so they are uncached.  In round 2, single-GPU batches that ran after
// virtual-shard runs had allocated and freed uncached records diverged from the oracle; round 5
// tied that class of divergence to freeing uncached allocations (below, g_special; DESIGN.md
// §5.2), so the uncached records are allocated once per process, after an L2 write-back, and
// never freed; everything else, virtual shards included, uses plain device memory.
// A pool of such sets, one per (device, concurrent engine): a second engine alive at the same
// time (or a second shard on the device) takes another set instead of falling back to cached
// memory.
struct UncachedRecords {
    int dev = -1;
    unsigned long long *ga = nullptr, *gb = nullptr, *gdone = nullptr;
    bool busy = false;
};
std::vector<UncachedRecords> g_urec;

// The same rule for the pending pivot rows U when they are not plain device memory (fine-grained
// across devices; uncached under the diagnostic switch): allocated once, kept for the process's
// lifetime and handed to later engines (best fit on the same device and flags), never freed.
// Round 5 found what the round-2/4 divergences share (profiles/r05_uncached_u_bisect.txt): W = 8
// virtual-shard solves with uncached U diverge from one shard only after earlier engines have
// freed such allocations -- the same code with every uncached U kept allocated was bit-exact in
// 12 of 12 solves, with them freed it diverged in 4 of 12 -- so no engine frees one.  The pool
// holds at most the largest set of such buffers alive at once, plus one buffer each time a solve
// needs a larger one than any free (a process solving one shape repeatedly reuses one set).  Pinned
// host buffers (acquire_pinned) live in the same pool.
struct SpecialBuf {
    int dev = -1;
    unsigned flags = 0;
    size_t bytes = 0;
    void *p = nullptr;
    bool busy = false;
};
std::vector<SpecialBuf> g_special;

void say(const char *s) {
    if (g_cfg.verbose) {
        printf("%s\n", s);
        fflush(stdout);
    }
}

inline size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

template <typename T>
T *dalloc(size_t count) {
    T *p = nullptr;
    if (count == 0) count = 1;
    SX_HIP(hipMalloc(reinterpret_cast<void **>(&p), count * sizeof(T)));
    return p;
}

// ------------------------------------------------------------------ TIMER CSV (chrono.cu:8-57)
// Same file names and format as the reference's -D TIMER build: header
// "vars,contraints,operation,elapsed_time", one row "rows,cols,op,us" per timed operation
// (rows = tableau width in the reference's counting, cols = m), one "solve" row per
// iteration of the pivot loop including the terminating one.  Enabled by
// simplex_set_timer_dir() or SIMPLEX_TIMER_DIR.
struct Chrono {
    FILE *f = nullptr;
    hipEvent_t a = nullptr, b = nullptr;

    bool on() const { return f != nullptr; }

    void open(int n, int m) {
        if (g_cfg.no_timer) return;
        std::string dir = g_cfg.timer_dir;
        if (dir.empty()) {
            const char *e = getenv("SIMPLEX_TIMER_DIR");
            if (e) dir = e;
        }
        if (dir.empty()) return;
        char name[96];
        if (g_cfg.benchmark) {
            snprintf(name, sizeof(name), "/benchmark_%d_%d.txt", n, m);
        } else {
            time_t t = time(nullptr);
            char ts[32];
            strftime(ts, sizeof(ts), "%Y%m%d%H%M%S.%d", localtime(&t));
            snprintf(name, sizeof(name), "/times_%s.txt", ts);
        }
        f = openFile((dir + name).c_str(), "w");
        fprintf(f, "vars,contraints,operation,elapsed_time\n");
        SX_HIP(hipEventCreate(&a));
        SX_HIP(hipEventCreate(&b));
    }
    void start(hipStream_t s, int rows, int cols, const char *op) {
        if (!f) return;
        fprintf(f, "%d,%d,%s,", rows, cols, op);
        SX_HIP(hipEventRecord(a, s));
    }
    void stop(hipStream_t s) {
        if (!f) return;
        SX_HIP(hipEventRecord(b, s));
        SX_HIP(hipEventSynchronize(b));
        float ms = 0.f;
        SX_HIP(hipEventElapsedTime(&ms, a, b));
        fprintf(f, "%f\n", ms * 1000.0f);
    }
    void row(int rows, int cols, const char *op, float ms) {
        if (f) fprintf(f, "%d,%d,%s,%f\n", rows, cols, op, ms * 1000.0f);
    }
    ~Chrono() {
        if (f) {
            fclose(f);
            (void)hipEventDestroy(a);
            (void)hipEventDestroy(b);
        }
    }
};

// Devices of a one-process multi-GPU engine ("Multi-GPU is internal: the caller
// still sees one synchronous call; the device list comes from SIMPLEX_GPUS"): simplex_set_gpus,
// else SIMPLEX_GPUS = "N" (devices 0..N-1) or a comma list ("0,1,2,3"; a device may repeat:
// several shards on one GPU).  Empty: one shard on the current device.
std::vector<int> shard_devices() {
    std::vector<int> v = g_cfg.gpus;
    if (v.empty()) {
        const char *e = getenv("SIMPLEX_GPUS");
        if (e == nullptr || *e == 0) return v;
        if (strchr(e, ',') == nullptr) {
            const int n = atoi(e);
            for (int i = 0; i < n; ++i) v.push_back(i);
        } else {
            for (const char *p = e; *p;) {
                v.push_back(atoi(p));
                const char *c = strchr(p, ',');
                if (c == nullptr) break;
                p = c + 1;
            }
        }
    }
    if (v.size() <= 1) return v;
    if ((int)v.size() > SX_MAXW) SX_FATAL("SIMPLEX_GPUS: at most 8 shards");
    int count = 0;
    SX_HIP(hipGetDeviceCount(&count));
    for (int d : v)
        if (d < 0 || d >= count) {
            char msg[128];
            snprintf(msg, sizeof(msg), "SIMPLEX_GPUS: device %d requested but %d visible", d, count);
            SX_FATAL(msg);
        }
    return v;
}

bool gpus_selftest(const std::vector<int> &devs);  // (below two_phase)
int gpus_check(const std::vector<int> &devs);

// the engine's own tableaux in 4x4 blocks (TLay::blk) unless SIMPLEX_BLOCKED=0 or
// simplex_set_blocked(0) selects row-major storage (the layout of callers' tableaux, tabular.h)
bool use_blocked() {
    if (g_cfg.blocked < 0) {
        const char *e = getenv("SIMPLEX_BLOCKED");
        return !(e && atoi(e) == 0);
    }
    return g_cfg.blocked != 0;
}

// makes `dev` current for its scope
struct DevGuard {
    int prev = -1;
    explicit DevGuard(int dev) {
        SX_HIP(hipGetDevice(&prev));
        if (dev != prev) SX_HIP(hipSetDevice(dev));
        else prev = -1;
    }
    ~DevGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// ------------------------------------------------------------------ shard + engine
struct Shard {
    int rank = 0;
    int row0 = 0;
    int rows = 0;
    double *T = nullptr;
    double *d = nullptr;
    double *d_save = nullptr;         // fused batch: d as the batch found it (restored after SX_HANG)
    double *dx = nullptr;             // RCCL ranks: this rank's objective-row slice, -0.0 elsewhere (gather_d)
    double *colE = nullptr;
    double *prow = nullptr;
    double *prow_send = nullptr;
    double *slot_send = nullptr;  // row-gather: per tile [TilePart header | winner row]
    double *slot_all = nullptr;
    double *U = nullptr;              // pending pivot rows [SX_KMAX][ld]
    int *perm = nullptr;              // slack compaction (Cols): logical slack -> stored offset [m]
    int *iperm = nullptr;             //   stored offset -> logical slack [m]
    int *ucol = nullptr;              //   row r -> the unswept slack column that is e_r, or -1 [m]
    int *urow = nullptr;              //   unswept slack k -> the row of its unit vector [m]
    int *nact = nullptr;              //   swept slack columns (the swept block's width past 1+n)
    DeactList *dlist = nullptr;       //   basic slacks moved out of the sweep (one shard)
    unsigned long long *dtag = nullptr;  // its scratch: stored slack offset -> (round, basic row) [m]
    unsigned dround = 0;                 //   rounds run
    int *dfail = nullptr;                //   slack -> 1 + the row whose check it failed [m]
    double *F = nullptr;              // pending row factors [rows][SX_KMAX]
    PivRec *recs = nullptr;           // pending pivot records [SX_KMAX]
    unsigned long long *PM = nullptr; // [rows] pending leaving-row slots (batch-tagged)
    unsigned long long *PM2 = nullptr; // [rows] the same for the second stage's slots
    double *coef = nullptr;
    double *gemv_local = nullptr;
    double *gemv_all = nullptr;
    double *rhs_local = nullptr;
    double *rhs_all = nullptr;
    int *base = nullptr;
    TilePart *enter_parts = nullptr;
    TilePart *tiles_local = nullptr;
    TilePart *tiles_all = nullptr;
    BatchChan *chan = nullptr;        // fused batch kernel: exit counter, abort word
    unsigned long long *ga = nullptr; // fused batch kernel: ratio-tile records (tagged granules)
    unsigned long long *gb = nullptr; // fused batch kernel: objective-tile records (tagged granules)
    unsigned long long *gdone = nullptr;  // multi-rank fused batch: batch-end done granules (one per rank)
    hipStream_t ss = nullptr;         // virtual shards: the stream its multi-rank fused batch runs on
    int dev = 0;                      // the device holding the shard's buffers
    hipStream_t s = nullptr;          // the engine's stream on that device (every per-shard operation)
    int urec = -1;                    // ga / gb / gdone: index of the uncached record set (g_urec), or -1
    bool fineU = false;               // U in fine-grained memory (peers on other devices write it)
    bool Upool = false;               // U is one of the process's kept allocations (g_special)
    DevState *st = nullptr;
};

class Engine {
  public:
    int n = 0, m = 0;
    int W = 1;             // total shards (ranks)
    bool rccl = false;     // true: one shard per process (collectives over RCCL unless ipc)
    bool ipc = false;      // one shard per process, peer buffers through caller-exchanged IPC handles only
    bool xchg = false;     // exchange path: tile allgather + pivot-row allreduce per pivot
    bool rowgather = false;  // exchange path variant: one allgather of tile winners with their rows
    size_t slot_stride = 0;  // doubles per row-gather slot (16-byte header + ld)
    int N1 = 0, N2 = 0, N = 0;
    bool alias = false;    // phase-1 artificial columns stored as their slack columns (sx_common.hpp Cols)
    bool compact = false;  // untouched slack columns kept past the swept block (sx_common.hpp Cols)
    int Ns1 = 0;           // stored columns in phase 1
    size_t ld = 0;         // full stored row width in doubles (U's row stride; T's without region B)
    TLay tl;               // T's storage regions (sx_common.hpp)
    int rpr = 0;           // rows per rank (multiple of 512)
    int slots = 0;         // argmin tiles / GEMV blocks per rank
    int device = 0;        // the primary device (shard 0's)
    hipStream_t s = nullptr;  // the engine stream on the primary device
    bool gpus_mode = false;   // one process, one shard per listed device (SIMPLEX_GPUS / simplex_set_gpus)
    bool multidev = false;    // ... on more than one device
    std::vector<int> shard_dev;            // gpus_mode: the device of each shard
    std::map<int, hipStream_t> dstream;    // the engine stream of every device in use (s on the primary)
    std::map<int, hipEvent_t> djoin;       // multidev: one join event per device stream
    std::vector<Shard> sh;
    const double **sum_srcs = nullptr;  // pinned host array of prow_send pointers (virtual ranks)
    DevState *st_host = nullptr;        // pinned: 2 poll slots
    hipEvent_t poll_ev[2] = {nullptr, nullptr};
    double *c_dev = nullptr;            // objective coefficients c (phase 2)
    long long phase_pivots[2] = {0, 0};
    // deferred pivots: the host numbers batches (ids never repeat, 0 is never used) and the
    // slots inside the current one; every batch ends with a sweep of the tableau
    unsigned batch_id = 1;  // 1 .. 2^15 - 1 (the granule tags keep 15 bits; see enqueue_sweep)
    int q_host = 0;
    bool batch_activated = false;  // the pending batch's fused kernel already activated its slack columns
    mutable bool wide_note = false;  // the verbose note "too wide for the fused batch" was printed
    unsigned long long *stamps = nullptr;  // diagnostic: in-kernel timestamps of the fused batch
    long long sweeps = 0;
    std::function<void(int)> on_pivot;  // DEBUG trace: called after every pivot (solver.cu:112-116)
    // split (not replicated) multi-rank batches may run fused: every shard's U is fine-grained, or no
    // shard's U can be written from another device (decided once, when the shards are allocated)
    bool split_ok = true;

    Engine(int n_, int m_, bool alias_ = true) : n(n_), m(m_) {
        N1 = 1 + n + 2 * m;
        N2 = 1 + n + m;
        N = N1;
        alias = alias_ && g_cfg.alias && m > 0;
        Ns1 = alias ? N2 : N1;
        ld = round_up((size_t)Ns1, 16);
        batch_id = (g_cfg.first_batch_id >= 1 && g_cfg.first_batch_id < SX_BATCH_IDS) ? g_cfg.first_batch_id : 1;
        std::vector<int> devs;  // one process, several GPUs: the device of every shard
        int alone_dev = -1;     // a device list that failed its self-check: every solve on its first device
        if (g_cfg.single_shard) {
            // one shard on this device
        } else if (g_cfg.ipc_world > 1) {
            rccl = ipc = true;
            W = g_cfg.ipc_world;
        } else if (g_cfg.dist && g_cfg.comm) {
            rccl = true;
            W = g_cfg.world;
        } else if ((devs = shard_devices()).size() > 1) {
            if (gpus_check(devs) != 0) {
                W = (int)devs.size();
                gpus_mode = true;
            } else {
                alone_dev = devs[0];  // (the list failed its self-check: its first device alone)
            }
        } else if (g_cfg.virtual_ranks > 1) {
            W = g_cfg.virtual_ranks;
        }
        xchg = W > 1 || g_cfg.force_exchange;
        slot_stride = ld + 2;
        int dev = 0;
        if (gpus_mode)
            SX_HIP(hipSetDevice(devs[0]));
        else if (alone_dev >= 0)
            SX_HIP(hipSetDevice(alone_dev));
        else if (g_cfg.device >= 0)
            SX_HIP(hipSetDevice(g_cfg.device));
        SX_HIP(hipGetDevice(&dev));
        device = dev;
        SX_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        dstream[device] = s;
        if (gpus_mode) {
            for (int d : devs) multidev = multidev || d != device;
            shard_dev = devs;
            if (multidev) open_devices();
        }
        rpr = (int)round_up((size_t)((m + W - 1) / W), SX_TILE);
        if (rpr == 0) rpr = SX_TILE;
        slots = rpr / SX_TILE;
        if ((long long)W * slots > SX_TILE) SX_FATAL("too many constraint tiles for the exact argmin tree");
        // Storage regions (sx_common.hpp TLay): with aliasing -- the precondition
        // of slack compaction -- region A holds the structural columns and the first capA stored
        // slack positions, region B the other slack positions, so the swept prefix of a row is
        // most of a row of A (dense streaming: 32768 x 9216 swept 5.7 TB/s with dense rows, 5.3
        // with rows 4.4x wider than the swept part, profiles/r02_sweep_row_stride.txt)
        tl.ldA = ld;
        tl.jB = Ns1;
        tl.blk = alias && use_blocked() ? 1 : 0;  // (callers' tableaux -- tabular.h, no aliasing -- stay row-major)
        if (alias && g_cfg.regions) {
            const int capA = g_cfg.regions >= 2 ? g_cfg.regions : std::max(4096, (m + 7) / 8);
            const int jB = (int)round_up((size_t)(1 + n + capA), SX_TILE);
            if (jB < Ns1) {
                tl.jB = jB;
                tl.ldA = (size_t)jB;
                tl.ldB = round_up((size_t)(Ns1 - jB), 16);
                tl.offB = (size_t)rpr * tl.ldA;  // every shard allocates rpr rows (peers index alike)
            }
        }
        // one allgather of (tile winner, row) beats two collectives while the rows are small
        const double slot_bytes = 8.0 * (double)slots * (double)slot_stride;
        rowgather = xchg && (g_cfg.exchange_mode == 2 || (g_cfg.exchange_mode == 0 && slot_bytes <= 1048576.0));
        std::vector<int> ranks;
        if (rccl)
            ranks.push_back(ipc ? g_cfg.ipc_rank : g_cfg.rank);
        else
            for (int k = 0; k < W; ++k) ranks.push_back(k);
        for (int k : ranks) {
            Shard x;
            x.rank = k;
            x.row0 = k * rpr;
            x.rows = m - x.row0;
            if (x.rows < 0) x.rows = 0;
            if (x.rows > rpr) x.rows = rpr;
            x.dev = gpus_mode ? shard_dev[(size_t)k] : device;
            x.s = dstream[x.dev];
            DevGuard g(x.dev);
            alloc_shard(x);
            sh.push_back(x);
        }
        if ((rccl && !ipc) || multidev)
            for (const auto &x : sh) split_ok = split_ok && x.fineU;
        if (!rccl && xchg) {
            // the shards' pivot-row contributions (pinned host memory: read by every device's kernel)
            sum_srcs = acquire_pinned<const double *>((size_t)W);
            for (int k = 0; k < W; ++k) sum_srcs[k] = sh[(size_t)k].prow_send;
        }
        st_host = acquire_pinned<DevState>(2);
        for (auto &e : poll_ev) SX_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        setup_peers();
    }

    // ---------------------------------------------------------------- one process, several devices
    // peer access between every pair of the shards' devices, one engine stream and one join event
    // per device
    void open_devices() {
        std::vector<int> ds;
        for (int d : shard_dev)
            if (std::find(ds.begin(), ds.end(), d) == ds.end()) ds.push_back(d);
        for (int a : ds) {
            DevGuard g(a);
            for (int b : ds) {
                if (a == b) continue;
                int can = 0;
                SX_HIP(hipDeviceCanAccessPeer(&can, a, b));
                if (!can) {
                    char msg[128];
                    snprintf(msg, sizeof(msg), "SIMPLEX_GPUS: device %d cannot access device %d's memory", a, b);
                    SX_FATAL(msg);
                }
                const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) SX_HIP(e);
                (void)hipGetLastError();
            }
            if (!dstream.count(a)) {
                hipStream_t st;
                SX_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
                dstream[a] = st;
            }
            hipEvent_t ev;
            SX_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            djoin[a] = ev;
        }
    }

    // every device stream waits for the work enqueued so far on all of them (the shards'
    // cross-device dependencies: collectives, gathers); a no-op on one device
    void join() {
        if (!multidev) return;
        for (auto &kv : dstream) {
            DevGuard g(kv.first);
            SX_HIP(hipEventRecord(djoin[kv.first], kv.second));
        }
        for (auto &kv : dstream) {
            DevGuard g(kv.first);
            for (auto &ev : djoin)
                if (ev.first != kv.first) SX_HIP(hipStreamWaitEvent(kv.second, ev.second, 0));
        }
    }

    // the host waits for every device stream
    void sync_all() {
        for (auto &kv : dstream) {
            DevGuard g(kv.first);
            SX_HIP(hipStreamSynchronize(kv.second));
        }
    }

    // ---------------------------------------------------------------- peer memory (multi-rank fused batch)
    PeerView pv;
    bool p2p = false;
    hipEvent_t ev_fork = nullptr;
    std::vector<hipEvent_t> ev_join;
    std::vector<void *> opened;  // peer allocations mapped through IPC

    void setup_peers() {
        std::memset(&pv, 0, sizeof(pv));
        if (ipc) return;  // the caller connects the peers (connect_peers)
        if (!xchg || W > SX_MAXW || g_cfg.p2p == 0) return;
        if (rccl && !(g_cfg.p2p == 1 || g_cfg.p2p_ready)) return;
        sync_all();
        // one process, several GPUs (SIMPLEX_GPUS): when the start-up self-check passes (or p2p is
        // forced); the batches run as one launch per device
        if (gpus_mode && g_cfg.p2p != 1 && !gpus_selftest(shard_dev)) return;
        // virtual shards: only when asked for (a test hook); their batches run as one launch
        // (mr_single_launch), or as W launches on W streams for W <= 3 (the engine stream + W
        // streams on 4 hardware queues)
        if (!rccl && !gpus_mode && (g_cfg.p2p != 1 || (W > 3 && !g_cfg.mr_single_launch))) return;
        if (!rccl) {  // shards of this process: every shard's buffers mapped here; one stream per shard
            for (auto &x : sh) {
                pv.T[x.rank] = x.T;
                pv.ga[x.rank] = x.ga;
                pv.gb[x.rank] = x.gb;
                pv.gdone[x.rank] = x.gdone;
                pv.U[x.rank] = x.U;
                pv.F[x.rank] = x.F;
                pv.d[x.rank] = x.d;
                if (multidev) continue;  // (one launch per device on its engine stream)
                SX_HIP(hipStreamCreateWithFlags(&x.ss, hipStreamNonBlocking));
                hipEvent_t e;
                SX_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
                ev_join.push_back(e);
            }
            if (!multidev) SX_HIP(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
            p2p = true;
            return;
        }
        // one shard per process: exchange IPC handles of the six buffers over RCCL, map the peers'
        // (a failure here is not fatal: every rank learns whether all mapped, and they all fall
        // back to the RCCL exchange together)
        std::vector<unsigned char> all((size_t)W * kHandles);
        int ok = export_handles(all.data() + (size_t)g_cfg.rank * kHandles);
        unsigned char *dev = dalloc<unsigned char>(all.size());
        SX_HIP(hipMemcpy(dev + (size_t)g_cfg.rank * kHandles, all.data() + (size_t)g_cfg.rank * kHandles, kHandles,
                         hipMemcpyHostToDevice));
        SX_NCCL(ncclAllGather(dev + (size_t)g_cfg.rank * kHandles, dev, kHandles, ncclUint8, g_cfg.comm, s));
        SX_HIP(hipMemcpyAsync(all.data(), dev, all.size(), hipMemcpyDeviceToHost, s));
        SX_HIP(hipStreamSynchronize(s));
        (void)hipFree(dev);
        ok = ok && map_peers(all.data(), g_cfg.rank);
        if (!all_ranks(ok)) {
            unmap_peers();
            if (g_cfg.verbose) say("peer memory unavailable: per-pivot RCCL exchange");
            return;
        }
        p2p = true;
    }

    // IPC handles of this process's seven exchanged buffers (T, ga, gb, gdone, U, d, F)
    static constexpr int kBufs = 7;
    static constexpr size_t kHandles = kBufs * sizeof(hipIpcMemHandle_t);
    int export_handles(unsigned char *out) {
        const Shard &x = sh[0];
        void *bufs[kBufs] = {x.T, x.ga, x.gb, x.gdone, x.U, x.d, x.F};
        int ok = 1;
        for (int k = 0; k < kBufs; ++k) {
            hipIpcMemHandle_t h;
            std::memset(&h, 0, sizeof(h));
            ok &= hipIpcGetMemHandle(&h, bufs[k]) == hipSuccess;
            std::memcpy(out + k * sizeof(h), &h, sizeof(h));
        }
        (void)hipGetLastError();
        return ok;
    }

    // map every other rank's buffers from `all` (W x kHandles bytes) into pv; false if any fails
    bool map_peers(const unsigned char *all, int me) {
        const Shard &x = sh[0];
        void *mine[kBufs] = {x.T, x.ga, x.gb, x.gdone, x.U, x.d, x.F};
        std::vector<void *> mapped((size_t)W * kBufs, nullptr);
        bool ok = true;
        for (int r = 0; r < W && ok; ++r)
            for (int k = 0; k < kBufs && ok; ++k) {
                if (r == me) {
                    mapped[(size_t)r * kBufs + k] = mine[k];
                    continue;
                }
                hipIpcMemHandle_t h;
                std::memcpy(&h, all + (size_t)r * kHandles + k * sizeof(h), sizeof(h));
                if (hipIpcOpenMemHandle(&mapped[(size_t)r * kBufs + k], h, hipIpcMemLazyEnablePeerAccess) == hipSuccess)
                    opened.push_back(mapped[(size_t)r * kBufs + k]);
                else
                    ok = false;
            }
        (void)hipGetLastError();
        if (!ok) return false;
        for (int r = 0; r < W; ++r) {
            void *const *p = &mapped[(size_t)r * kBufs];
            pv.T[r] = static_cast<const double *>(p[0]);
            pv.ga[r] = static_cast<unsigned long long *>(p[1]);
            pv.gb[r] = static_cast<unsigned long long *>(p[2]);
            pv.gdone[r] = static_cast<unsigned long long *>(p[3]);
            pv.U[r] = static_cast<double *>(p[4]);
            pv.d[r] = static_cast<double *>(p[5]);
            pv.F[r] = static_cast<const double *>(p[6]);
        }
        return true;
    }

    void unmap_peers() {
        for (void *p : opened) (void)hipIpcCloseMemHandle(p);
        opened.clear();
        std::memset(&pv, 0, sizeof(pv));
    }

    // 1 on every rank iff `ok` on every rank (an RCCL min-allreduce; RCCL ranks only)
    bool all_ranks(int ok) {
        int *dv = dalloc<int>(1);
        SX_HIP(hipMemcpy(dv, &ok, sizeof(int), hipMemcpyHostToDevice));
        SX_NCCL(ncclAllReduce(dv, dv, 1, ncclInt, ncclMin, g_cfg.comm, s));
        int r = 0;
        SX_HIP(hipMemcpyAsync(&r, dv, sizeof(int), hipMemcpyDeviceToHost, s));
        SX_HIP(hipStreamSynchronize(s));
        (void)hipFree(dv);
        return r != 0;
    }

    void close_peers() {
        if (opened.empty()) return;
        unmap_peers();
        if (ipc) return;  // (the caller keeps every process alive until all have unmapped)
        // every rank has unmapped before any rank frees what the others mapped
        int *one = dalloc<int>(1);
        SX_NCCL(ncclAllReduce(one, one, 1, ncclInt, ncclSum, g_cfg.comm, s));
        (void)hipStreamSynchronize(s);
        (void)hipFree(one);
    }

    ~Engine() {
        sync_all();
        close_peers();
        for (auto &x : sh)
            if (x.ss) (void)hipStreamDestroy(x.ss);
        if (ev_fork) (void)hipEventDestroy(ev_fork);
        for (auto &e : ev_join)
            if (e) (void)hipEventDestroy(e);
        for (auto &x : sh) {
            DevGuard g(x.dev);
            free_shard(x);
        }
        if (sum_srcs) release_special(sum_srcs);
        if (c_dev) (void)hipFree(c_dev);
        if (u_bad) (void)hipFree(u_bad);
        if (st_host) release_special(st_host);
        for (auto &e : poll_ev)
            if (e) (void)hipEventDestroy(e);
        for (auto &kv : djoin) {
            DevGuard g(kv.first);
            (void)hipEventDestroy(kv.second);
        }
        for (auto &kv : dstream) {
            DevGuard g(kv.first);
            (void)hipStreamDestroy(kv.second);
        }
    }

    // doubles of a shard's tableau allocation (the blocked layout: whole 16-row strips)
    size_t t_doubles(size_t rows_alloc) const {
        if (tl.blk) rows_alloc = round_up(rows_alloc, 16);
        return tl.jB < Ns1 ? tl.offB + (size_t)rpr * tl.ldB : rows_alloc * tl.ldA;
    }

    // a free uncached record set on `dev` (allocated, after an L2 write-back, the first time)
    static int acquire_uncached_records(int dev, hipStream_t st) {
        for (size_t i = 0; i < g_urec.size(); ++i)
            if (g_urec[i].dev == dev && !g_urec[i].busy) {
                g_urec[i].busy = true;
                return (int)i;
            }
        UncachedRecords u;
        u.dev = dev;
        sx_launch_l2_writeback(st);
        SX_HIP(hipStreamSynchronize(st));
        SX_HIP(hipExtMallocWithFlags(reinterpret_cast<void **>(&u.ga), sx_batch_granules_a() * 8, hipDeviceMallocUncached));
        SX_HIP(hipExtMallocWithFlags(reinterpret_cast<void **>(&u.gb), sx_batch_granules_b() * 8, hipDeviceMallocUncached));
        SX_HIP(hipExtMallocWithFlags(reinterpret_cast<void **>(&u.gdone), SX_MAXW * 8, hipDeviceMallocUncached));
        u.busy = true;
        g_urec.push_back(u);
        return (int)g_urec.size() - 1;
    }

    // a free special allocation (g_special) of >= bytes on `dev` with `flags`, allocated after an L2
    // write-back when none is free
    static void *acquire_special(int dev, unsigned flags, size_t bytes, hipStream_t st) {
        int best = -1;
        for (size_t i = 0; i < g_special.size(); ++i) {
            const SpecialBuf &b = g_special[i];
            if (b.dev == dev && b.flags == flags && !b.busy && b.bytes >= bytes &&
                (best < 0 || b.bytes < g_special[(size_t)best].bytes))
                best = (int)i;
        }
        if (best >= 0) {
            g_special[(size_t)best].busy = true;
            return g_special[(size_t)best].p;
        }
        SpecialBuf b;
        b.dev = dev;
        b.flags = flags;
        b.bytes = bytes;
        sx_launch_l2_writeback(st);
        SX_HIP(hipStreamSynchronize(st));
        SX_HIP(hipExtMallocWithFlags(&b.p, bytes, flags));
        b.busy = true;
        g_special.push_back(b);
        return b.p;
    }
    // pinned host memory (the engine's state mirror, the per-pivot exchange's source list) under the
    // same rule: allocated once, reused by later engines, never freed (every
    // non-plain allocation, not only U)
    static constexpr unsigned kPinnedHost = 0xffffffffu;
    template <typename T>
    static T *acquire_pinned(size_t count) {
        const size_t bytes = count * sizeof(T);
        int best = -1;
        for (size_t i = 0; i < g_special.size(); ++i) {
            const SpecialBuf &b = g_special[i];
            if (b.flags == kPinnedHost && !b.busy && b.bytes >= bytes &&
                (best < 0 || b.bytes < g_special[(size_t)best].bytes))
                best = (int)i;
        }
        if (best >= 0) {
            g_special[(size_t)best].busy = true;
            return static_cast<T *>(g_special[(size_t)best].p);
        }
        SpecialBuf b;
        b.flags = kPinnedHost;
        b.bytes = bytes;
        SX_HIP(hipHostMalloc(&b.p, bytes, hipHostMallocDefault));
        b.busy = true;
        g_special.push_back(b);
        return static_cast<T *>(b.p);
    }
    static void release_special(void *p) {
        for (auto &b : g_special)
            if (b.p == p) b.busy = false;
    }

    // (on the shard's device)
    void alloc_shard(Shard &x) {
        const size_t rows_alloc = x.rows > 0 ? (size_t)x.rows : 1;
        x.T = dalloc<double>(t_doubles(rows_alloc));
        // d: plain device memory (no rank writes another's).  U: other ranks write the pending pivot
        // rows into it over xGMI (system-scope stores) in the multi-rank batch, and this rank's sweep
        // reads them with plain loads in a later kernel.  Across devices it is fine-grained memory
        // (coherent with the peers' system-scope writes by construction, not through this device's
        // L2: DESIGN.md §5); on one device, or when forced off, plain device memory.
        x.d = dalloc<double>(round_up((size_t)N1, 16));
        int fu = g_cfg.fine_u;
        if (fu < 0) {  // (SIMPLEX_FINE_PIVOT_ROWS=0/1/2 overrides the default, as simplex_set_fine_pivot_rows)
            const char *e = getenv("SIMPLEX_FINE_PIVOT_ROWS");
            if (e) fu = atoi(e);
        }
        // (with the replicated objective every rank forms the whole pivot row itself and no peer
        // writes U, once every batch of the solve fits that way)
        // (test hook, fu == 2: U of exchanging shards in uncached memory -- the allocation of the
        // round-4/5 divergence, DESIGN.md §5.2, kept reachable for tests/test_gpu_empty_shards.py)
        const bool uncU = fu == 2 && xchg;
        x.fineU = fu == 1 || (fu < 0 && ((rccl && !ipc) || multidev) && !repl_always());
        const unsigned uflags = uncU ? hipDeviceMallocUncached : x.fineU ? hipDeviceMallocFinegrained : 0u;
        x.Upool = uflags != 0u;
        if (x.Upool)  // (kept for the process, g_special)
            x.U = static_cast<double *>(acquire_special(x.dev, uflags, (size_t)SX_KMAX * ld * sizeof(double), x.s));
        else
            x.U = dalloc<double>((size_t)SX_KMAX * ld);
        x.d_save = dalloc<double>(round_up((size_t)N1, 16));
        x.colE = dalloc<double>(rows_alloc);
        x.prow = dalloc<double>(ld);
        if (xchg) x.prow_send = dalloc<double>(ld);
        if (rowgather) {
            x.slot_send = dalloc<double>((size_t)slots * slot_stride);
            x.slot_all = dalloc<double>((size_t)W * slots * slot_stride);
            std::vector<double> init((size_t)slots * slot_stride, 0.0);
            for (int k = 0; k < slots; ++k) {
                TilePart *h = reinterpret_cast<TilePart *>(init.data() + (size_t)k * slot_stride);
                h->v = 1.7976931348623157e308;
                h->idx = -1;
                h->elig = 0;
            }
            SX_HIP(hipMemcpy(x.slot_send, init.data(), sizeof(double) * init.size(), hipMemcpyHostToDevice));
        }
        x.F = dalloc<double>(round_up(rows_alloc, 16) * SX_KMAX);  // (sx_fidx: whole 16-row strips)
        x.recs = dalloc<PivRec>(SX_KMAX);
        x.PM = dalloc<unsigned long long>(rows_alloc);
        x.PM2 = dalloc<unsigned long long>(rows_alloc);
        SX_HIP(hipMemsetAsync(x.U, 0, (size_t)SX_KMAX * ld * sizeof(double), x.s));
        SX_HIP(hipMemsetAsync(x.F, 0, round_up(rows_alloc, 16) * SX_KMAX * sizeof(double), x.s));
        SX_HIP(hipMemsetAsync(x.recs, 0, SX_KMAX * sizeof(PivRec), x.s));
        SX_HIP(hipMemsetAsync(x.PM, 0, rows_alloc * sizeof(unsigned long long), x.s));
        SX_HIP(hipMemsetAsync(x.PM2, 0, rows_alloc * sizeof(unsigned long long), x.s));
        x.coef = dalloc<double>(rows_alloc);
        x.rhs_local = dalloc<double>(rpr);
        if (xchg) x.rhs_all = dalloc<double>((size_t)W * rpr);
        x.base = dalloc<int>(m);
        x.enter_parts = dalloc<TilePart>(SX_TILE);
        x.chan = dalloc<BatchChan>(1);
        if ((rccl && !ipc) || multidev) {
            // polled while other GPUs write them: one of the process's uncached record sets
            x.urec = acquire_uncached_records(x.dev, x.s);
            x.ga = g_urec[(size_t)x.urec].ga;
            x.gb = g_urec[(size_t)x.urec].gb;
            x.gdone = g_urec[(size_t)x.urec].gdone;
        } else {
            // one device (virtual shards, processes sharing a GPU): plain memory, sc1 hand-offs
            x.ga = dalloc<unsigned long long>(sx_batch_granules_a());
            x.gb = dalloc<unsigned long long>(sx_batch_granules_b());
            if (xchg) x.gdone = dalloc<unsigned long long>(SX_MAXW);
        }
        if (x.gdone) SX_HIP(hipMemsetAsync(x.gdone, 0, SX_MAXW * 8, x.s));
        SX_HIP(hipMemsetAsync(x.chan, 0, sizeof(BatchChan), x.s));
        SX_HIP(hipMemsetAsync(x.ga, 0, sx_batch_granules_a() * sizeof(unsigned long long), x.s));
        SX_HIP(hipMemsetAsync(x.gb, 0, sx_batch_granules_b() * sizeof(unsigned long long), x.s));
        x.tiles_local = dalloc<TilePart>(slots);
        if (xchg) x.tiles_all = dalloc<TilePart>((size_t)W * slots);
        x.st = dalloc<DevState>(1);
        SX_HIP(hipMemsetAsync(x.T, 0, t_doubles(rows_alloc) * sizeof(double), x.s));
        SX_HIP(hipMemsetAsync(x.d, 0, round_up((size_t)N1, 16) * sizeof(double), x.s));
        SX_HIP(hipMemsetAsync(x.prow, 0, ld * sizeof(double), x.s));
        // padding tile entries must read (DBL_MAX, -1, not eligible)
        std::vector<TilePart> pad((size_t)W * slots);
        for (auto &t : pad) {
            t.v = 1.7976931348623157e308;
            t.idx = -1;
            t.elig = 0;
        }
        SX_HIP(hipMemcpy(x.tiles_local, pad.data(), sizeof(TilePart) * slots, hipMemcpyHostToDevice));
        if (xchg)
            SX_HIP(hipMemcpy(x.tiles_all, pad.data(), sizeof(TilePart) * pad.size(), hipMemcpyHostToDevice));
    }

    void free_shard(Shard &x) {
        if (x.urec >= 0) {  // the process's uncached records stay allocated (g_urec)
            x.ga = x.gb = x.gdone = nullptr;
            g_urec[(size_t)x.urec].busy = false;
            x.urec = -1;
        }
        if (x.Upool) {  // (U stays allocated for later engines, g_special)
            release_special(x.U);
            x.U = nullptr;
            x.Upool = false;
        }
        for (void *p : {(void *)x.T, (void *)x.d, (void *)x.d_save, (void *)x.dx, (void *)x.colE, (void *)x.prow, (void *)x.prow_send,
                        (void *)x.slot_send, (void *)x.slot_all, (void *)x.U, (void *)x.F, (void *)x.recs, (void *)x.PM, (void *)x.PM2,
                        (void *)x.coef, (void *)x.gemv_local, (void *)x.gemv_all, (void *)x.rhs_local,
                        (void *)x.rhs_all, (void *)x.base, (void *)x.enter_parts, (void *)x.tiles_local, (void *)x.chan,
                        (void *)x.ga, (void *)x.gb, (void *)x.gdone, (void *)x.perm, (void *)x.iperm,
                        (void *)x.ucol, (void *)x.urow, (void *)x.nact, (void *)x.dlist, (void *)x.dtag, (void *)x.dfail,
                        (void *)x.tiles_all, (void *)x.st})
            if (p) (void)hipFree(p);
    }

    // ---------------------------------------------------------------- phase-1 tableau
    // fillTableu (twoPhaseMethod.cu:145-200): each shard copies only its rows of A.  (b and c
    // live on the primary device; the other devices' kernels read them through peer access.)
    void build_phase1(const problem_t *P) {
        double *b_dev = dalloc<double>(m);
        SX_HIP(hipMemcpyAsync(b_dev, P->knownTermsVector, sizeof(double) * m, hipMemcpyHostToDevice, s));
        SX_HIP(hipStreamSynchronize(s));
        for (auto &x : sh) {
            DevGuard g(x.dev);
            double *A_local = nullptr;
            if (x.rows > 0 && n > 0) {
                A_local = dalloc<double>((size_t)x.rows * n);
                SX_HIP(hipMemcpy2DAsync(A_local, sizeof(double) * x.rows, P->constraintsMatrix + x.row0,
                                        sizeof(double) * m, sizeof(double) * x.rows, n, hipMemcpyHostToDevice, x.s));
            }
            sx_launch_build_rows(x.T, x.rows, x.row0, tl, n, m, Ns1, A_local, b_dev, x.s);
            sx_launch_init_vectors(x.d, N1, n, m, x.base, x.s);
            SX_HIP(hipStreamSynchronize(x.s));
            if (A_local) (void)hipFree(A_local);
        }
        (void)hipFree(b_dev);
        if (!c_dev) {
            c_dev = dalloc<double>(n);
            if (n > 0)
                SX_HIP(hipMemcpy(c_dev, P->objectiveFunction, sizeof(double) * n, hipMemcpyHostToDevice));
        }
        bool nonneg = true;  // no row negated (k_fill_rows negates b < -eps; b < 0 is stricter)
        for (int i = 0; i < m; ++i) nonneg = nonneg && !(P->knownTermsVector[i] < 0.0);
        set_compact(nonneg);
    }

    // the same tableau as build_phase1(generateRandomProblem(n, m, seed, lo, hi)), synthesised
    // on the device: every shard generates only its own rows (jump-ahead XORWOW)
    void build_phase1_generated(unsigned seed, int lo, int hi, int rand_kind) {
        uint32_t sd[3];
        sx_crt_seeds(seed, rand_kind, sd);
        double *b_dev = dalloc<double>(m);
        sx_launch_gen_vector(sd[0], 0, m, lo, hi, b_dev, s);
        if (!c_dev) c_dev = dalloc<double>(n);
        sx_launch_gen_vector(sd[1], 0, n, lo, hi, c_dev, s);
        SX_HIP(hipStreamSynchronize(s));
        for (auto &x : sh) {
            DevGuard g(x.dev);
            sx_launch_gen_rows(sd[2], n, m, x.row0, x.rows, lo, hi, x.T, tl, nullptr, x.s);
            sx_launch_build_rows(x.T, x.rows, x.row0, tl, n, m, Ns1, nullptr, b_dev, x.s);
            sx_launch_init_vectors(x.d, N1, n, m, x.base, x.s);
        }
        sync_all();
        (void)hipFree(b_dev);
        set_compact(lo >= 0);  // b in [lo, hi]: no row negated
    }

    // ---------------------------------------------------------------- collectives
    // Shards of this process (virtual shards, or one per GPU): device copies between their
    // buffers, after a join of the device streams (and before the next, so every device sees
    // the result); RCCL ranks: one collective on the engine stream.
    void allgather_tiles() {
        if (rccl) {
            Shard &x = sh[0];
            SX_NCCL(ncclAllGather(x.tiles_local, x.tiles_all, sizeof(TilePart) * slots, ncclUint8, g_cfg.comm, s));
            return;
        }
        join();
        for (auto &dst : sh) {
            DevGuard g(dst.dev);
            for (auto &src : sh)
                SX_HIP(hipMemcpyAsync(dst.tiles_all + (size_t)src.rank * slots, src.tiles_local,
                                      sizeof(TilePart) * slots, hipMemcpyDeviceToDevice, dst.s));
        }
        join();
    }

    void allgather_slots() {
        const size_t count = (size_t)slots * slot_stride;
        if (rccl) {
            Shard &x = sh[0];
            SX_NCCL(ncclAllGather(x.slot_send, x.slot_all, count, ncclDouble, g_cfg.comm, s));
            return;
        }
        join();
        for (auto &dst : sh) {
            DevGuard g(dst.dev);
            for (auto &src : sh)
                SX_HIP(hipMemcpyAsync(dst.slot_all + (size_t)src.rank * count, src.slot_send, sizeof(double) * count,
                                      hipMemcpyDeviceToDevice, dst.s));
        }
        join();
    }

    void allreduce_prow() {
        if (rccl) {
            Shard &x = sh[0];
            SX_NCCL(ncclAllReduce(x.prow_send, x.prow, cols(N).Ns, ncclDouble, ncclSum, g_cfg.comm, s));
            return;
        }
        join();
        for (auto &dst : sh) {
            DevGuard g(dst.dev);
            sx_launch_sum_rows(dst.prow, sum_srcs, W, cols(N).Ns, dst.s);
        }
        join();
    }

    void allgather_doubles(double *Shard::*local, double *Shard::*all, size_t count) {
        if (rccl) {
            Shard &x = sh[0];
            SX_NCCL(ncclAllGather(x.*local, x.*all, count, ncclDouble, g_cfg.comm, s));
            return;
        }
        join();
        for (auto &dst : sh) {
            DevGuard g(dst.dev);
            for (auto &src : sh)
                SX_HIP(hipMemcpyAsync(dst.*all + (size_t)src.rank * count, src.*local, sizeof(double) * count,
                                      hipMemcpyDeviceToDevice, dst.s));
        }
        join();
    }

    // The objective row after fused multi-rank batches: each rank kept only its own slice current
    // (the columns of its objective tiles, and d[0] on the rank holding tile 0; sx_kernels.hip
    // batch_mr_body); this
    // hands every rank the whole row.  RCCL ranks: a sum all-reduce of rows that hold the rank's
    // slice and -0.0 elsewhere (x + -0.0 == x for every x, -0.0 included: exact); shards of this
    // process: device copies of the slices.  IPC test ranks: the caller's simplex_session_sync_d.
    bool d_split = false;

    // logical columns [j0, j1) of rank k's slice; d[0] belongs to the rank whose objective tiles
    // start with tile 0 (own0) -- not always rank 0: a rank can have no objective tile when the
    // phase has fewer 512-column tiles than ranks
    void d_slice(int k, int &j0, int &j1, bool &own0) const {
        const int NBg = (N - 1 + SX_TILE - 1) / SX_TILE;
        const int tb0 = (int)((long long)k * NBg / W), tb1 = (int)((long long)(k + 1) * NBg / W);
        j0 = 1 + tb0 * SX_TILE;
        j1 = std::min(1 + tb1 * SX_TILE, N);
        if (j0 > j1) j0 = j1;
        own0 = tb0 == 0 && tb1 > 0;
    }

    void gather_d() {
        if (!d_split) return;
        // IPC ranks (a test mode) cannot gather here: the row is whole only after every process has
        // called simplex_session_sync_d.  A kernel that needs it before then would read a stale
        // split row -- refuse loudly instead (and keep d_split, so reads stay refused too).
        if (ipc) SX_FATAL("IPC session: the objective row is split between ranks (simplex_session_sync_d first)");
        d_split = false;
        if (rccl) {
            Shard &x = sh[0];
            if (!x.dx) x.dx = dalloc<double>(round_up((size_t)N1, 16));
            int j0, j1;
            bool own0;
            d_slice(x.rank, j0, j1, own0);
            sx_launch_d_contrib(x.d, x.dx, N, j0, j1, own0 ? 1 : 0, s);
            SX_NCCL(ncclAllReduce(x.dx, x.d, N, ncclDouble, ncclSum, g_cfg.comm, s));
            return;
        }
        join();
        for (auto &dst : sh) {
            DevGuard g(dst.dev);
            for (auto &src : sh) {
                if (src.rank == dst.rank) continue;
                int j0, j1;
                bool own0;
                d_slice(src.rank, j0, j1, own0);
                if (j1 > j0)
                    SX_HIP(hipMemcpyAsync(dst.d + j0, src.d + j0, sizeof(double) * (j1 - j0), hipMemcpyDeviceToDevice,
                                          dst.s));
                if (own0) SX_HIP(hipMemcpyAsync(dst.d, src.d, sizeof(double), hipMemcpyDeviceToDevice, dst.s));
            }
        }
        join();
    }

    // IPC test ranks: write this rank's slice into every peer's objective row (the caller
    // barriers the processes before and after)
    void publish_d_ipc() {
        if (!ipc) return;
        d_split = false;
        Shard &x = sh[0];
        int j0, j1;
        bool own0;
        d_slice(x.rank, j0, j1, own0);
        for (int k = 0; k < W; ++k) {
            if (k == x.rank || pv.d[k] == nullptr) continue;
            if (j1 > j0)
                SX_HIP(hipMemcpyAsync(pv.d[k] + j0, x.d + j0, sizeof(double) * (j1 - j0), hipMemcpyDeviceToDevice, s));
            if (own0) SX_HIP(hipMemcpyAsync(pv.d[k], x.d, sizeof(double), hipMemcpyDeviceToDevice, s));
        }
        SX_HIP(hipStreamSynchronize(s));
    }

    // ---------------------------------------------------------------- objective GEMV
    // updateObjectiveFunction (gaussian.cu:132-162), deterministic blocked order.
    void update_objective(int width) {
        gather_d();
        const Cols c = cols(width);
        const size_t part = (size_t)slots * c.Ns;
        for (auto &x : sh) {
            DevGuard g(x.dev);
            if (!x.gemv_local) x.gemv_local = dalloc<double>((size_t)slots * Ns1);
            if (xchg && !x.gemv_all) x.gemv_all = dalloc<double>((size_t)W * slots * Ns1);
            SX_HIP(hipMemsetAsync(x.gemv_local, 0, part * sizeof(double), x.s));
            sx_launch_coef(x.d, x.base, x.row0, x.rows, x.coef, x.s);
            sx_launch_gemv_partials(x.T, x.rows, tl, c.Ns, x.coef, x.gemv_local, x.s);
        }
        if (xchg) allgather_doubles(&Shard::gemv_local, &Shard::gemv_all, part);
        const int nblk = (m + SX_TILE - 1) / SX_TILE;
        for (auto &x : sh) {
            DevGuard g(x.dev);
            sx_launch_gemv_apply(x.d, cols(width, x), xchg ? x.gemv_all : x.gemv_local, nblk, x.s);
        }
    }

    void phase2_costs() {
        gather_d();
        for (auto &x : sh) {
            DevGuard g(x.dev);
            sx_launch_phase2_costs(x.d, n, m, c_dev, x.s);
        }
    }

    // logical width of a phase -> stored columns
    Cols cols(int width) const {
        Cols c;
        c.N = width;
        const bool a = alias && width == N1;
        c.Ns = a ? Ns1 : width;
        c.art0 = a ? 1 + n + m : 0x7fffffff;
        c.shift = m;
        c.s0 = 1 + n;
        c.perm = nullptr;
        return c;
    }
    // the same, with the shard's slack permutation (device pointer) when compacting
    Cols cols(int width, const Shard &x) const {
        Cols c = cols(width);
        if (compact) c.perm = x.perm;
        return c;
    }

    // Slack compaction (sx_common.hpp Cols): valid while every slack column is built as +e_k
    // -- no row negated by the b < 0 quirk (its -0.0 entries would let a pivot flip the sign
    // of a zero) -- and phase 1 stores artificials as their slacks.  Off for a caller's
    // tableau (upload).
    void set_compact(bool on) {
        on = on && alias && m > 0 && g_cfg.compact != 0;
        if (on) {
            std::vector<int> id((size_t)m);
            for (int k = 0; k < m; ++k) id[k] = k;
            for (auto &x : sh) {
                DevGuard g(x.dev);
                if (!x.perm) {
                    x.perm = dalloc<int>(m);
                    x.iperm = dalloc<int>(m);
                    x.ucol = dalloc<int>(m);
                    x.urow = dalloc<int>(m);
                    x.nact = dalloc<int>(1);
                    x.dlist = dalloc<DeactList>(1);
                    x.dtag = dalloc<unsigned long long>(m);
                    x.dfail = dalloc<int>(m);
                }
                SX_HIP(hipMemcpyAsync(x.perm, id.data(), sizeof(int) * m, hipMemcpyHostToDevice, x.s));
                SX_HIP(hipMemcpyAsync(x.iperm, id.data(), sizeof(int) * m, hipMemcpyHostToDevice, x.s));
                SX_HIP(hipMemcpyAsync(x.ucol, id.data(), sizeof(int) * m, hipMemcpyHostToDevice, x.s));
                SX_HIP(hipMemcpyAsync(x.urow, id.data(), sizeof(int) * m, hipMemcpyHostToDevice, x.s));
                SX_HIP(hipMemsetAsync(x.nact, 0, sizeof(int), x.s));
                SX_HIP(hipMemsetAsync(x.dlist, 0, sizeof(DeactList), x.s));
                SX_HIP(hipMemsetAsync(x.dtag, 0, sizeof(unsigned long long) * m, x.s));
                SX_HIP(hipMemsetAsync(x.dfail, 0, sizeof(int) * m, x.s));
                x.dround = 0;
            }
            sync_all();
        }
        compact = on;
    }

    // swept slack columns (m when not compacting)
    int active_slacks() {
        if (!compact) return m;
        int v = 0;
        SX_HIP(hipMemcpyAsync(&v, sh[0].nact, sizeof(int), hipMemcpyDeviceToHost, s));
        SX_HIP(hipStreamSynchronize(s));
        return v;
    }

    // ---------------------------------------------------------------- one pivot
    SweepCfg sweep_cfg(int batch) const {
        // The vector sweep steps 4 rows at 32 pivots per sweep (config 3: 138 us), 2 at 16 (127 us)
        // and stores write-through (sc1; faster at every size from 32 MiB to 512 MiB, 4096 x 8192
        // 98 vs 110 us, profiles/r02_sweep_sc1_sizes.txt) -- which also keeps no row of the tableau
        // dirty in an L2 of this device when peer ranks read leaving rows from it (system-scope
        // loads over xGMI); the matrix-core sweep stores write-through too.
        SweepCfg c;
        c.batch = batch;
        // (a two-stage batch: the matrix-core sweep, the only one holding SX_KMAX slots; one stage:
        // the matrix cores too by default -- with the strip-major factors the vector sweep's
        // per-row factor loads are scalar loads 128 B apart, config 2/3/5 no faster on the vector
        // units, profiles/r03_onestage_mfma_ab.txt)
        c.mfma = batch > SX_HMAX ? 1 : (g_cfg.sweep_mfma >= 0 ? g_cfg.sweep_mfma : 1);
        return c;
    }

    // pivots per sweep: the configured batch (1 while tracing every pivot); two stages (SX_KMAX)
    // only in the fused batches -- one shard's and the peer-memory multi-rank one; the per-pivot
    // kernels and the vector sweep hold one stage (run_phase caps it again when the batch is not
    // fused)
    // Default: two stages when the tableau has >= 4096 rows -- the second stage's longer chains
    // (+0.7 to +1.4 us per pivot, the first stage's 32 pending pivots applied on the fly) cost
    // less than the sweep they save (same box: config 5 27.6 -> 15.4 us of sweep per pivot,
    // 23.7k -> 33.4k pivots/s; config 3 3.80 -> 2.88 us, 71.6k -> 72.9k; profiles/r03_flayout_ab.txt)
    int batch_size() const {
        if (on_pivot) return 1;
        const int want = g_cfg.batch > 0 ? g_cfg.batch : (m >= 4096 ? SX_KMAX : SX_HMAX);
        if (g_cfg.mr_two_stage < 0) {
            const char *e = getenv("SIMPLEX_MR_STAGES");
            g_cfg.mr_two_stage = (e && atoi(e) == 1) ? 0 : 1;
        }
        const bool two_stage = g_cfg.fused != 0 && ((!xchg && sh.size() == 1) || (xchg && p2p && g_cfg.mr_two_stage));
        const int cap = two_stage ? SX_KMAX : SX_HMAX;
        return std::max(1, std::min(want, cap));
    }

    Pending pending(const Shard &x) const {
        Pending p;
        p.U = x.U;
        p.F = x.F;
        p.recs = x.recs;
        p.PM = x.PM;
        p.PM2 = x.PM2;
        p.batch = batch_id;
        p.q = q_host;
        return p;
    }

    // pass 1 of the entering argmin for the first pivot of a phase (later pivots get it
    // from k_pivot_row)
    void enqueue_enter_partials() {
        gather_d();
        for (auto &x : sh) {
            DevGuard g(x.dev);
            sx_launch_enter(x.d, N - 1, x.enter_parts, x.st, x.s);
        }
    }

    // one pivot into slot q_host of the current batch: ratio test + selection, the pivot
    // row, the objective row and the next entering variable.  The tableau is not touched.
    void enqueue_pivot() {
        gather_d();
        for (auto &x : sh) {
            DevGuard g(x.dev);
            sx_launch_ratio_select(x.T, x.rows, x.row0, ld, tl, x.tiles_local, x.colE, x.st, x.base, !xchg,
                                   rowgather ? x.slot_send : nullptr, slot_stride, cols(N, x), pending(x), x.s);
        }
        if (rowgather) {
            allgather_slots();
            for (auto &x : sh) {
                DevGuard g(x.dev);
                sx_launch_select_gathered(x.slot_all, slot_stride, W * slots, x.base, x.st, pending(x), x.s);
            }
        } else if (xchg) {
            allgather_tiles();
            for (auto &x : sh) {
                DevGuard g(x.dev);
                sx_launch_select_row(x.T, x.rows, x.row0, ld, tl, cols(N, x), x.tiles_all, W * slots, x.prow_send, x.base,
                                     x.st, pending(x), x.s);
            }
            allreduce_prow();
        }
        for (auto &x : sh) {
            DevGuard g(x.dev);
            const double *pb = rowgather ? x.slot_all : (xchg ? x.prow : nullptr);
            sx_launch_pivot_row(x.T, x.rows, x.row0, ld, tl, cols(N, x), x.d, pb, rowgather ? slot_stride : 0, x.colE, x.st,
                                pending(x), x.enter_parts, x.s);
        }
        ++q_host;
    }

    // a whole batch of up to k pivots in one resident launch (one shard, no exchange)
    bool fused_ok(int k) const {
        if (g_cfg.fused == 0 || on_pivot) return false;
        if (!xchg) {
            if ((N - 1 + SX_TILE - 1) / SX_TILE > sx_batch_obj_tile_limit() && g_cfg.verbose && !wide_note) {
                wide_note = true;  // (the width limit of the one-shard fused batch)
                fprintf(stderr, "simplex: %d objective tiles exceed the fused batch's %d (N - 1 > %d): per-pivot path\n",
                        (N - 1 + SX_TILE - 1) / SX_TILE, sx_batch_obj_tile_limit(), sx_batch_obj_tile_limit() * SX_TILE);
            }
            return sh.size() == 1 && sx_batch_fits(sh[0].rows, cols(N), k);
        }
        if (!p2p) return false;
        const int NBg = (N - 1 + SX_TILE - 1) / SX_TILE;
        if (repl_now(k)) return true;
        if (!split_ok) return false;  // (peers would write a plain U across devices: the per-pivot path)
        return sx_batch_mr_fits(slots, (NBg + W - 1) / W, k, mr_grids());
    }

    // ranks resident together on one device (virtual shards: all of them)
    int mr_grids() const {
        if (rccl) return 1;
        if (!gpus_mode) return std::max(1, W);  // (virtual shards: all on this device)
        int grids = 1;
        std::map<int, int> per_dev;
        for (int d : shard_dev) grids = std::max(grids, ++per_dev[d]);
        return grids;
    }
    // The replicated objective: every rank runs every objective tile, so each
    // rank decides the entering variable from its own records and forms the whole pivot row in
    // its own U -- the only cross-rank hand-offs of a pivot are the ratio tiles' winners and the
    // leaving row read from its owner.  Default across devices (RCCL ranks, a device list on
    // several GPUs), where the objective hop is an xGMI hop; forced on or off by
    // simplex_set_replicated_objective.  Used for a batch when its grid (slots + every objective
    // tile per rank) fits, else the split objective.
    // In IPC mode (one process per rank, peers connected by the caller) d is gathered only by
    // simplex_session_sync_d, so a replicated batch could start from a stale split row: never there.
    // When some shard's U is plain memory while its peers sit on other devices (split_ok false: the
    // allocation-time decision, alloc_shard), only replicated batches -- no peer writes U -- may run
    // fused, whatever simplex_set_replicated_objective says now.
    bool repl_mode() const {
        if (W < 2 || ipc) return false;
        if (!split_ok) return true;
        if (g_cfg.repl_obj == 0) return false;
        return g_cfg.repl_obj > 0 || rccl || multidev;
    }
    bool repl_now(int k) const {
        return repl_mode() && sx_batch_mr_fits(slots, (N - 1 + SX_TILE - 1) / SX_TILE, k, mr_grids());
    }
    // ... for every batch of this engine (phase 1 is the widest)
    bool repl_always() const {
        return repl_mode() && g_cfg.fused != 0 &&
               sx_batch_mr_fits(slots, (N1 - 1 + SX_TILE - 1) / SX_TILE, SX_KMAX, mr_grids());
    }

    void enqueue_batch(int k) {
        if (q_host != 0) SX_FATAL("fused batch inside a started batch");
        ++g_cfg.fused_batches;
        if (g_cfg.inject_hang >= 0 && g_cfg.inject_hang-- == 0)  // test hook: this batch aborts
            for (auto &x : sh) {
                DevGuard g(x.dev);
                if (g_cfg.inject_slot < 0)
                    SX_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(&x.chan->abort_w), 1u, 1, x.s));
                else
                    SX_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(&x.chan->inject_q),
                                             (unsigned)g_cfg.inject_slot + 1u, 1, x.s));
            }
        if (!xchg) {
            Shard &x = sh[0];
            sx_launch_batch(x.T, x.rows, ld, tl, cols(N, x), x.d, x.d_save, x.base, x.st, pending(x), k, x.chan, x.ga, x.gb,
                            stamps, compact ? x.perm : nullptr, x.iperm, x.ucol, x.urow, x.nact, m, s);
            batch_activated = compact;  // (its last block did k_activate's work)
            q_host = k;
            return;
        }
        const bool rp = repl_now(k);
        if (rp) gather_d();  // (a replicated batch starts from the whole row on every rank)
        d_split = !rp;       // (split multi-rank batches keep only each rank's own slice of d current)
        const int NBgk = (N - 1 + SX_TILE - 1) / SX_TILE;
        auto tb_of = [&](int rank, int &tb0, int &tb1) {
            tb0 = rp ? 0 : (int)((long long)rank * NBgk / W);
            tb1 = rp ? NBgk : (int)((long long)(rank + 1) * NBgk / W);
        };
        if (!rccl && (g_cfg.mr_single_launch || multidev)) {
            // shards of this process: the ranks on one GPU as ONE launch (all of them for virtual
            // shards; one launch per GPU when each shard has its own), so a device's ranks are
            // resident together whenever the grid fits; they hand off through each other's
            // buffers exactly as RCCL ranks do through peer memory
            std::map<int, std::vector<MrLaunchRank>> by_dev;
            for (size_t i = 0; i < sh.size(); ++i) {
                Shard &x = sh[i];
                MrLaunchRank q;
                q.T = x.T;
                q.rows = x.rows;
                q.row0 = x.row0;
                q.rank = x.rank;
                tb_of(x.rank, q.tb0, q.tb1);
                q.repl = rp ? 1 : 0;
                q.perm = compact ? x.perm : nullptr;
                q.d = x.d;
                q.d_save = x.d_save;
                q.base = x.base;
                q.st = x.st;
                q.pd = pending(x);
                q.chan = x.chan;
                q.ga = x.ga;
                q.gb = x.gb;
                q.gdone = x.gdone;
                by_dev[x.dev].push_back(q);
            }
            const unsigned long long timeout = multidev ? 200000000ull : 100000000ull;  // 2 s / 1 s at 100 MHz
            for (auto &kv : by_dev) {
                DevGuard g(kv.first);
                sx_launch_batch_mr_multi(kv.second.data(), (int)kv.second.size(), W, rpr, ld, tl, cols(N), batch_id, k,
                                         slots, pv, timeout, dstream[kv.first]);
            }
        } else {
            // every rank's batch runs at once (virtual shards: one stream each, forked from and
            // joined back into the engine stream); the ranks hand off through peer memory
            const unsigned long long timeout = rccl ? 200000000ull : 100000000ull;  // 2 s / 1 s at 100 MHz
            if (!rccl) SX_HIP(hipEventRecord(ev_fork, s));
            for (size_t i = 0; i < sh.size(); ++i) {
                Shard &x = sh[i];
                hipStream_t xs = s;
                if (!rccl) {
                    xs = x.ss;
                    SX_HIP(hipStreamWaitEvent(xs, ev_fork, 0));
                }
                int tb0, tb1;
                tb_of(x.rank, tb0, tb1);
                sx_launch_batch_mr(x.T, x.rows, x.row0, rpr, ld, tl, cols(N, x), x.d, x.d_save, x.base, x.st, pending(x), k,
                                   slots, W, x.rank, tb0, tb1, rp ? 1 : 0, x.chan, x.ga, x.gb, x.gdone, pv, timeout, xs);
                if (!rccl) SX_HIP(hipEventRecord(ev_join[i], xs));
            }
            if (!rccl)
                for (auto &e : ev_join) SX_HIP(hipStreamWaitEvent(s, e, 0));
        }
        q_host = k;
    }

    // apply the batch's pivots to the tableau (a no-op kernel when none was selected) and
    // start a new batch
    // rec_shard0: the sweep record target (sx_set_sweep_record) is meant for shard 0's sweep
    void enqueue_sweep(hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr, bool rec_shard0 = false) {
        if (q_host == 0) return;
        const SweepCfg cfg = sweep_cfg(q_host);
        const int rev = (int)(sweeps & 1);  // alternate the sweep direction (Infinity-Cache reuse)
        // the slack exchanges first (each shard's own buffers), so the events bracket the
        // sweeps alone (ev0 / ev1 on the engine stream: shard 0's sweep)
        if (compact && !batch_activated)
            for (auto &x : sh) {
                DevGuard g(x.dev);
                sx_launch_activate(x.perm, x.iperm, x.ucol, x.urow, x.nact, m, x.T, x.rows, x.row0, ld, tl, 1 + n, pending(x), x.st,
                                   q_host, x.s);
            }
        if (check_u_on()) check_pivot_rows();
        if (ev0) SX_HIP(hipEventRecord(ev0, s));
        for (auto &x : sh) {
            DevGuard g(x.dev);
            sx_launch_sweep(x.T, x.rows, x.row0, ld, tl, cols(N).Ns, compact ? x.nact : nullptr, 1 + n, pending(x), x.st, rev, cfg,
                            x.s);
            if (rec_shard0) sx_set_sweep_record(nullptr);  // (only shard 0's sweep records)
        }
        if (rec_shard0) sx_set_sweep_record(nullptr);
        if (ev1) SX_HIP(hipEventRecord(ev1, s));
        // one shard, every g_cfg.deact sweeps: the swept slacks whose columns are exactly their unit
        // vectors leave the swept block.  (Not on several shards: each sees only its rows of a column,
        // and the shards would have to agree on every check -- a column that entered keeps the
        // residuals a_k - fl(a_k / p) p where they are not 0)
        if (g_cfg.deact < 0) {
            const char *e = getenv("SIMPLEX_DEACTIVATE");
            g_cfg.deact = e ? (atoi(e) > 0 ? atoi(e) : 0) : 8;
        }
        if (compact && W == 1 && g_cfg.deact > 0 && (sweeps + 1) % g_cfg.deact == 0 && m <= 65536) {
            Shard &x = sh[0];
            sx_launch_deactivate(x.perm, x.iperm, x.ucol, x.urow, x.nact, x.base, n, m, cols(N).art0 != 0x7fffffff, x.T,
                                 x.rows, x.row0, tl, 1 + n, x.dtag, ++x.dround, true, x.dfail, x.dlist, x.s);
        }
        ++sweeps;
        q_host = 0;
        batch_activated = false;
        if (++batch_id >= SX_BATCH_IDS) wrap_batch_ids();
    }

    // the pivot-row check (diagnostic): shards of this process only -- RCCL ranks' peers start their
    // next batch, which writes into this rank's U, while a check here would still read
    unsigned long long *u_bad = nullptr;
    bool check_u_on() const {
        if (g_cfg.check_u < 0) {
            const char *e = getenv("SIMPLEX_CHECK_PIVOT_ROWS");
            g_cfg.check_u = e && atoi(e) == 1 ? 1 : 0;
        }
        return g_cfg.check_u == 1 && W > 1 && !rccl && q_host > 0;
    }
    void check_pivot_rows() {
        DevGuard g(device);
        PeerView v;
        std::memset(&v, 0, sizeof(v));
        for (auto &x : sh) v.U[x.rank] = x.U;
        if (!u_bad) {
            u_bad = dalloc<unsigned long long>(1);
            SX_HIP(hipMemsetAsync(u_bad, 0, sizeof(unsigned long long), s));
        }
        join();
        sx_launch_check_u(v, W, ld, cols(N).Ns, sh[0].st, batch_id, u_bad, s);
        unsigned long long bad = 0;
        SX_HIP(hipMemcpyAsync(&bad, u_bad, sizeof(bad), hipMemcpyDeviceToHost, s));
        SX_HIP(hipMemsetAsync(u_bad, 0, sizeof(unsigned long long), s));
        SX_HIP(hipStreamSynchronize(s));
        join();
        g_cfg.u_mismatches += (long long)bad;
    }

    // The granule tags keep 15 bits of the batch id ([id | slot (6) | payload (11)],
    // sx_kernels.hip make_tag) and PM[i] the whole id: before ids repeat, every id-tagged word
    // is cleared (0 is never an id), once per 32767 batches (about a million pivots).
    void wrap_batch_ids() {
        batch_id = 1;
        for (auto &x : sh) {
            DevGuard g(x.dev);
            SX_HIP(hipMemsetAsync(x.PM, 0, sizeof(unsigned long long) * (x.rows > 0 ? (size_t)x.rows : 1), x.s));
            SX_HIP(hipMemsetAsync(x.PM2, 0, sizeof(unsigned long long) * (x.rows > 0 ? (size_t)x.rows : 1), x.s));
            SX_HIP(hipMemsetAsync(x.ga, 0, sx_batch_granules_a() * sizeof(unsigned long long), x.s));
            SX_HIP(hipMemsetAsync(x.gb, 0, sx_batch_granules_b() * sizeof(unsigned long long), x.s));
            if (x.gdone) SX_HIP(hipMemsetAsync(x.gdone, 0, SX_MAXW * sizeof(unsigned long long), x.s));
        }
        // peer ranks write into these records: no rank starts its next batch before every rank
        // has cleared its own (an RCCL all-reduce behind the memsets on every rank; the shards of
        // this process: a join of the device streams)
        if (rccl && !ipc) all_ranks(1);
        join();
        sync_all();
    }

    void reset_state(long long max_pivots) {
        enqueue_sweep();  // never leave pivots of an earlier call unapplied
        DevState init;
        std::memset(&init, 0, sizeof(init));
        init.status = SX_NOT_ENDED;
        init.e = -1;
        init.r = -1;
        init.e_next = -1;
        init.max_pivots = max_pivots;
        for (auto &x : sh) {
            DevGuard g(x.dev);
            SX_HIP(hipMemcpyAsync(x.st, &init, sizeof(init), hipMemcpyHostToDevice, x.s));
        }
        sync_all();
    }

    DevState read_state() {
        DevState out;
        SX_HIP(hipMemcpyAsync(&out, sh[0].st, sizeof(out), hipMemcpyDeviceToHost, s));
        SX_HIP(hipStreamSynchronize(s));
        return out;
    }

    // solve (solver.cu:128-149): pivots until the phase ends.  Batches of pivots are
    // enqueued back to back; the host polls the status of the batch before the last one,
    // so the device never waits on the host.  Kernels of a finished phase return at once.
    int run_phase(int width, long long max_pivots, long long *pivots, Chrono *ch = nullptr) {
        N = width;
        reset_state(max_pivots);
        enqueue_enter_partials();
        int K = batch_size();
        const bool timed = ch && ch->on();
        std::vector<hipEvent_t> it_ev;  // TIMER CSV: one event pair per loop iteration
        if (on_pivot) {  // DEBUG: one pivot at a time, tableau printed after each
            for (;;) {
                enqueue_pivot();
                enqueue_sweep();
                if (read_state().status != SX_NOT_ENDED) break;
                on_pivot(width);
            }
        }
        // batches of K pivots + one sweep; the host polls the status of the batch before the
        // last one, so the device never waits on the host
        bool fused = !timed && fused_ok(K);
        if (!fused) K = std::min(K, SX_HMAX);
        int hangs = 0;
        long long k = 0;
        for (; !on_pivot; ++k) {
            if (fused) enqueue_batch(K);
            for (int b = 0; b < K && !fused; ++b) {
                if (timed) {
                    hipEvent_t e0, e1;
                    SX_HIP(hipEventCreate(&e0));
                    SX_HIP(hipEventCreate(&e1));
                    SX_HIP(hipEventRecord(e0, s));
                    enqueue_pivot();
                    if (b == K - 1) enqueue_sweep();  // the batch's sweep counts to its last pivot
                    SX_HIP(hipEventRecord(e1, s));
                    it_ev.push_back(e0);
                    it_ev.push_back(e1);
                } else {
                    enqueue_pivot();
                }
            }
            enqueue_sweep();
            const int slot = (int)(k & 1);
            SX_HIP(hipMemcpyAsync(st_host + slot, sh[0].st, sizeof(DevState), hipMemcpyDeviceToHost, s));
            SX_HIP(hipEventRecord(poll_ev[slot], s));
            if (k >= 1) {
                SX_HIP(hipEventSynchronize(poll_ev[slot ^ 1]));
                const int st = st_host[slot ^ 1].status;
                if (st == SX_HANG) {
                    // a fused batch's hand-off wait timed out (every rank sees it at the same
                    // batch): restore the state it found, re-run it on the per-pivot path
                    recover_hang(K);
                    if (++hangs >= 2) {  // not twice more: stay on the per-pivot path
                        fused = false;
                        K = std::min(K, SX_HMAX);
                    }
                    if (read_state().status != SX_NOT_ENDED) break;
                    k = -1;  // restart the lagged polling
                    continue;
                }
                if (st != SX_NOT_ENDED) break;
            }
        }
        if (!ipc) gather_d();  // (IPC ranks: the caller's simplex_session_sync_d)
        sync_all();  // (one synchronous call: every device's work is done)
        DevState f = read_state();
        if (timed) {
            const size_t iters = std::min(it_ev.size() / 2, (size_t)f.pivots + 1);
            for (size_t i = 0; i < iters; ++i) {
                float ms = 0.f;
                SX_HIP(hipEventElapsedTime(&ms, it_ev[2 * i], it_ev[2 * i + 1]));
                ch->row(width, m, "solve", ms);
            }
            for (auto e : it_ev) (void)hipEventDestroy(e);
        }
        if (pivots) *pivots = f.pivots;
        return f.status;
    }

    // After SX_HANG: the aborted batch changed neither T (its sweep found no pivot to apply),
    // the basis (written only by a completed batch) nor the state (only the status); its
    // objective row is restored from d_save.  The batch behind it saw the SX_HANG status and
    // did nothing.  The batch is then re-run on the per-pivot path, under fresh batch ids.
    // (Multi-rank batches: each rank restores its own slice -- the entries its threads saved --
    // and the whole row is then gathered, so no rank depends on a peer's aborted batch.)
    void recover_hang(int K) {
        sync_all();
        ++g_cfg.hang_recoveries;
        const int ne = SX_NOT_ENDED;
        for (auto &x : sh) {
            DevGuard g(x.dev);
            SX_HIP(hipMemcpyAsync(x.d, x.d_save, sizeof(double) * N, hipMemcpyDeviceToDevice, x.s));
            SX_HIP(hipMemcpyAsync(&x.st->status, &ne, sizeof(int), hipMemcpyHostToDevice, x.s));
        }
        for (int b = 0; b < K; ++b) {  // (the first gathers d; a two-stage batch: two sweeps)
            enqueue_pivot();
            if (q_host == SX_HMAX) enqueue_sweep();
        }
        enqueue_sweep();
        sync_all();
    }

    double read_d0() {
        double v = 0.0;
        SX_HIP(hipMemcpyAsync(&v, sh[0].d, sizeof(double), hipMemcpyDeviceToHost, s));
        SX_HIP(hipStreamSynchronize(s));
        return v;
    }

    void read_base(int *out) {
        SX_HIP(hipMemcpyAsync(out, sh[0].base, sizeof(int) * m, hipMemcpyDeviceToHost, s));
        SX_HIP(hipStreamSynchronize(s));
    }

    // the whole objective row d[0, width) (logical columns)
    void read_d(std::vector<double> &out, int width) {
        gather_d();
        sync_all();
        out.assign((size_t)width, 0.0);
        SX_HIP(hipMemcpyAsync(out.data(), sh[0].d, sizeof(double) * width, hipMemcpyDeviceToHost, s));
        SX_HIP(hipStreamSynchronize(s));
    }

    void write_base(const int *in) {
        for (auto &x : sh) {
            DevGuard g(x.dev);
            SX_HIP(hipMemcpyAsync(x.base, in, sizeof(int) * m, hipMemcpyHostToDevice, x.s));
        }
        sync_all();
    }

    // RHS column of all rows (for the solution, getSolution twoPhaseMethod.cu:116-128)
    void read_rhs(std::vector<double> &out) {
        out.assign(m, 0.0);
        for (auto &x : sh) {
            DevGuard g(x.dev);
            sx_launch_gather_rhs(x.T, x.rows, tl, x.rhs_local, x.s);
        }
        if (xchg) {
            allgather_doubles(&Shard::rhs_local, &Shard::rhs_all, rpr);
            SX_HIP(hipMemcpyAsync(out.data(), sh[0].rhs_all, sizeof(double) * m, hipMemcpyDeviceToHost, s));
        } else {
            SX_HIP(hipMemcpyAsync(out.data(), sh[0].rhs_local, sizeof(double) * m, hipMemcpyDeviceToHost, s));
        }
        SX_HIP(hipStreamSynchronize(s));
    }

    // rows of the whole tableau (virtual or single shard only), logical columns: for tests
    // and printing (aliased artificial columns are expanded from their slack columns)
    void download(double *T_host, size_t ld_host, int width, double *d_host, bool local_rows = false) {
        gather_d();
        sync_all();
        const Cols c = cols(width);
        std::vector<double> tmp;
        std::vector<int> perm;
        if (compact) {
            perm.resize((size_t)m);
            SX_HIP(hipMemcpyAsync(perm.data(), sh[0].perm, sizeof(int) * m, hipMemcpyDeviceToHost, s));
            SX_HIP(hipStreamSynchronize(s));
        }
        const int s0 = 1 + n;
        for (auto &x : sh) {
            if (x.rows <= 0 || T_host == nullptr) continue;  // (null: the objective row alone)
            tmp.assign((size_t)x.rows * c.Ns, 0.0);
            const int wa = std::min(c.Ns, tl.jB);  // region A's columns, then region B's
            DevGuard g(x.dev);
            if (tl.blk) {
                // blocked storage: rows converted to row-major on the device, a chunk at a time
                const int chunk = (int)std::max<size_t>(16, std::min<size_t>((size_t)x.rows, (64u << 20) / (8 * (size_t)c.Ns)));
                double *buf = dalloc<double>((size_t)chunk * c.Ns);
                for (int i0 = 0; i0 < x.rows; i0 += chunk) {
                    const int nr = std::min(chunk, x.rows - i0);
                    sx_launch_rows_out(x.T, tl, i0, nr, c.Ns, buf, x.s);
                    SX_HIP(hipMemcpyAsync(tmp.data() + (size_t)i0 * c.Ns, buf, sizeof(double) * nr * c.Ns,
                                          hipMemcpyDeviceToHost, x.s));
                }
                SX_HIP(hipStreamSynchronize(x.s));
                (void)hipFree(buf);
            } else {
                SX_HIP(hipMemcpy2DAsync(tmp.data(), c.Ns * sizeof(double), x.T, tl.ldA * sizeof(double),
                                        wa * sizeof(double), x.rows, hipMemcpyDeviceToHost, x.s));
                if (wa < c.Ns)
                    SX_HIP(hipMemcpy2DAsync(tmp.data() + wa, c.Ns * sizeof(double), x.T + tl.offB,
                                            tl.ldB * sizeof(double), (c.Ns - wa) * sizeof(double), x.rows,
                                            hipMemcpyDeviceToHost, x.s));
            }
            SX_HIP(hipStreamSynchronize(x.s));
            for (int i = 0; i < x.rows; ++i) {
                double *dst = T_host + (size_t)((local_rows ? 0 : x.row0) + i) * ld_host;
                const double *src = tmp.data() + (size_t)i * c.Ns;
                for (int j = 0; j < width; ++j) {
                    const int k = c.map(j);
                    dst[j] = src[(compact && k >= s0) ? s0 + perm[k - s0] : k];
                }
            }
        }
        if (d_host) SX_HIP(hipMemcpyAsync(d_host, sh[0].d, sizeof(double) * width, hipMemcpyDeviceToHost, s));
        SX_HIP(hipStreamSynchronize(s));
    }

    // logical columns in; with aliasing only the stored columns are taken (the caller's
    // artificial columns must equal the slack columns, checked by the callers below)
    void upload(const double *T_host, size_t ld_host, int width, const double *d_host, const int *base_host,
                bool local_rows = false) {
        set_compact(false);  // a caller's tableau: any column may be touched
        d_split = false;
        const Cols c = cols(width);
        for (auto &x : sh) {
            DevGuard g(x.dev);
            if (x.rows > 0) {
                const double *src = T_host + (size_t)(local_rows ? 0 : x.row0) * ld_host;
                const int wa = std::min(c.Ns, tl.jB);  // region A's columns, then region B's
                if (tl.blk) {
                    // blocked storage: row-major chunks to the device, placed by a kernel
                    const int chunk =
                        (int)std::max<size_t>(16, std::min<size_t>((size_t)x.rows, (64u << 20) / (8 * (size_t)c.Ns)));
                    double *buf = dalloc<double>((size_t)chunk * c.Ns);
                    for (int i0 = 0; i0 < x.rows; i0 += chunk) {
                        const int nr = std::min(chunk, x.rows - i0);
                        SX_HIP(hipMemcpy2DAsync(buf, c.Ns * sizeof(double), src + (size_t)i0 * ld_host,
                                                ld_host * sizeof(double), c.Ns * sizeof(double), nr,
                                                hipMemcpyHostToDevice, x.s));
                        sx_launch_rows_in(x.T, tl, i0, nr, c.Ns, 0, buf, c.Ns, x.s);
                    }
                    SX_HIP(hipStreamSynchronize(x.s));
                    (void)hipFree(buf);
                } else {
                    SX_HIP(hipMemcpy2DAsync(x.T, tl.ldA * sizeof(double), src, ld_host * sizeof(double),
                                            wa * sizeof(double), x.rows, hipMemcpyHostToDevice, x.s));
                    if (wa < c.Ns)
                        SX_HIP(hipMemcpy2DAsync(x.T + tl.offB, tl.ldB * sizeof(double), src + wa,
                                                ld_host * sizeof(double), (c.Ns - wa) * sizeof(double), x.rows,
                                                hipMemcpyHostToDevice, x.s));
                }
            }
            if (d_host) SX_HIP(hipMemcpyAsync(x.d, d_host, sizeof(double) * width, hipMemcpyHostToDevice, x.s));
            if (base_host) SX_HIP(hipMemcpyAsync(x.base, base_host, sizeof(int) * m, hipMemcpyHostToDevice, x.s));
        }
        sync_all();
    }
};

// true when a caller's phase-1-width tableau has every artificial column bit-identical to
// its slack column (so the aliased storage represents it exactly)
static bool artificial_equals_slack(const double *T, long long rows, long long N, long long ld, long long n,
                                    long long m) {
    if (n < 0 || m <= 0 || N != 1 + n + 2 * m) return false;
    for (long long i = 0; i < rows; ++i) {
        const double *row = T + i * ld;
        if (std::memcmp(row + 1 + n, row + 1 + n + m, sizeof(double) * (size_t)m) != 0) return false;
    }
    return true;
}
static bool artificial_equals_slack(const double *T, long long m, long long N, long long ld) {
    return artificial_equals_slack(T, m, N, ld, N - 1 - 2 * m, m);
}

// tabular_t <-> engine
std::map<const tabular_t *, Engine *> g_tabs;

// tabular.cu:41-98 print(): one line per tableau column (the reference stores the transpose):
// the m constraint entries, then the objective entry; the base vector last
void print_tableau(FILE *out, Engine &E, int width) {
    if (E.rccl) return;  // the rows of other ranks are not here
    const int m = E.m;
    std::vector<double> T((size_t)m * width), d(width);
    std::vector<int> base(m);
    E.download(T.data(), width, width, d.data());
    E.read_base(base.data());
    fprintf(out, "\n--------------- Tabular --------------\n");
    for (int j = 0; j < width; ++j) {
        for (int i = 0; i < m; ++i) fprintf(out, "%.2lf\t", T[(size_t)i * width + j]);
        fprintf(out, "\t|\t %.11lf\n", d[j]);
        if (j == 0) fprintf(out, "\n");
    }
    fprintf(out, "Base\n");
    for (int i = 0; i < m; ++i) fprintf(out, "%d\t", base[i]);
    fflush(out);
}

bool debug_on() {
    if (g_cfg.debug < 0) g_cfg.debug = getenv("SIMPLEX_DEBUG") ? 1 : 0;
    return g_cfg.debug > 0;
}

// The reference's entry points return only FEASIBLE / INFEASIBLE / UNBOUNDED / DEGENERATE
// (twoPhaseMethod.h:5-8; solve: FEASIBLE / UNBOUNDED, solver.cu:119-125); every other failure
// prints and exits (error.cu:5-12).  The engine-only outcomes follow that convention there
// (twoPhaseMethodEx keeps them as statuses).
int public_status(int st) {
    if (st == SX_NUMERIC_FAIL) SX_FATAL("simplex: the ratio test found no leaving row although a pivot is eligible");
    if (st == SX_HANG) SX_FATAL("simplex: a fused-batch hand-off between GPUs timed out");
    return st;
}

// ------------------------------------------------------------------ the two-phase driver
double g_phase_seconds[2] = {0.0, 0.0};  // wall time of the last solve's pivot loops (P1, P2)
std::vector<double> g_last_d;             // the last solve's final objective row (its last phase's width)

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int two_phase(problem_t *P, double *solution, double *opt, int *base_out, long long *pivots_out,
              long long max_pivots) {
    const int n = P->vars, m = P->constraints;
    Engine E(n, m);
    Chrono ch;
    ch.open(n, m);
    long long p1 = 0, p2 = 0;
    int status;
    // phase1 (twoPhaseMethod.cu:225-283)
    say("Phase 1: Filling Tableau");
    ch.start(E.s, E.N1, m, "fillTableau");
    E.build_phase1(P);
    ch.stop(E.s);
    say("Phase 1: Resetting out-of-base variables");
    if (debug_on()) {
        fprintf(stdout, "\nTableu nella situazione iniziale\n");
        print_tableau(stdout, E, E.N1);
        E.on_pivot = [&E](int w) { print_tableau(stdout, E, w); };
    }
    ch.start(E.s, E.N1, m, "gauss1");
    E.update_objective(E.N1);
    ch.stop(E.s);
    if (debug_on()) {
        fprintf(stdout, "\nTableu dopo l'eliminazione di gauss\n");
        print_tableau(stdout, E, E.N1);
    }
    say("Phase 1: Solving auxiliary problem");
    g_phase_seconds[0] = g_phase_seconds[1] = 0.0;
    double t0 = now_s();
    const int st1 = E.run_phase(E.N1, max_pivots, &p1, &ch);  // return value ignored by the reference (:258)
    g_phase_seconds[0] = now_s() - t0;
    if (debug_on()) {
        fprintf(stdout, "\nTableu dopo il lancio del primo solver\n");
        print_tableau(stdout, E, E.N1);
    }
    const double d0 = E.read_d0();
    std::vector<int> base(m);
    if (st1 == SX_PIVOT_CAP) {
        status = SX_PIVOT_CAP;
    } else if (st1 == SX_NUMERIC_FAIL || st1 == SX_HANG) {
        status = st1;
    } else if (compare(d0) < 0) {
        status = INFEASIBLE;  // :265-268
    } else {
        ch.start(E.s, E.N1, m, "checkDegeneracy");
        E.read_base(base.data());
        status = FEASIBLE;  // checkDegeneracy (:206-223)
        for (int i = 0; i < m; ++i)
            if (base[i] >= n + m && base[i] < n + 2 * m) status = DEGENERATE;
        ch.stop(E.s);
    }
    E.read_base(base.data());
    if (status != FEASIBLE) E.read_d(g_last_d, E.N1);
    if (status == FEASIBLE) {
        // phase2 (:285-356): drop the artificial columns, costs -c / 0, d[0] kept
        say("Phase 2: Filling costs vector with the original one");
        ch.start(E.s, E.N2, m, "costsVector");
        E.phase2_costs();
        ch.stop(E.s);
        say("Phase 2: Resetting out-of-base variables");
        ch.start(E.s, E.N2, m, "gauss2");
        E.update_objective(E.N2);
        ch.stop(E.s);
        say("Phase 2: Solving original problem");
        t0 = now_s();
        status = E.run_phase(E.N2, max_pivots, &p2, &ch);
        g_phase_seconds[1] = now_s() - t0;
        if (debug_on()) {
            fprintf(stdout, "\nTableu dopo seconda esecuzione del solver\n");
            print_tableau(stdout, E, E.N2);
        }
        E.read_base(base.data());
        E.read_d(g_last_d, E.N2);
        if (status == FEASIBLE) {
            // getSolutionHost (:370-383)
            ch.start(E.s, E.N2, m, "solution");
            const double z = E.read_d0();
            std::vector<double> rhs;
            E.read_rhs(rhs);
            if (opt) *opt = z;
            if (solution) {
                for (int j = 0; j < n; ++j) solution[j] = 0.0;
                for (int i = 0; i < m; ++i)
                    if (base[i] < n) solution[base[i]] = rhs[i];
            }
            ch.stop(E.s);
        }
    }
    if (base_out) std::memcpy(base_out, base.data(), sizeof(int) * m);
    if (pivots_out) {
        pivots_out[0] = p1;
        pivots_out[1] = p2;
    }
    return status;
}

// A small instance solved with the multi-rank fused batch over peer memory -- in one-stage (32) and
// two-stage (64-pivot) batches -- with the per-pivot exchange, and on one shard of this device
// alone (the reference answer).  The instance gives each of the W shards 512 rows (m = 512 W, rows
// per shard round_up(m / W, 512) = 512), so every rank sweeps, owns leaving rows and writes and
// reads peer pivot rows during the check (W = 2: m = 1100 -- 1318 + 23 pivots, phases ending
// mid-batch -- as before).  Returns 2 when both multi-shard paths give the one-shard answer bit for
// bit (and the fused path ran without a hand-off timing out), 1 when only the per-pivot exchange
// does, 0 when the per-pivot exchange does not either (the shards must not be used: one device).
// ref_dev: the device of the one-shard reference solve (-1: the current one; a SIMPLEX_GPUS list: its
// first device).  With peer-memory batches switched off (simplex_set_p2p(0)) only the per-pivot
// exchange is checked (2 solves instead of 4).
int selftest_solves(int W, int ref_dev) {
    const int sm = W > 2 ? 512 * W : 1100;
    problem_t *P = generateRandomProblem(300, sm, 300 * 100 + sm, 1, 100);
    const int n = P->vars, m = P->constraints;
    const int save = g_cfg.p2p, save_batch = g_cfg.batch, save_dev = g_cfg.device;
    const bool check_p2p = g_cfg.p2p != 0;
    const bool save_nt = g_cfg.no_timer, save_single = g_cfg.single_shard;
    g_cfg.no_timer = true;  // (timing would switch the solves to the per-pivot path; no CSVs either)
    struct Answer {
        std::vector<double> x;
        std::vector<int> base;
        long long piv[2] = {0, 0};
        double z = 0.0;
        int st = 0;
    };
    auto solve = [&](int p2p, int batch) {
        Answer a;
        a.x.assign(n, 0.0);
        a.base.assign(m, 0);
        g_cfg.p2p = p2p;
        g_cfg.batch = batch;
        a.st = two_phase(P, a.x.data(), &a.z, a.base.data(), a.piv, -1);
        return a;
    };
    auto same = [&](const Answer &a, const Answer &b) {
        return a.st == b.st && a.st != SX_HANG && a.piv[0] == b.piv[0] && a.piv[1] == b.piv[1] &&
               std::memcmp(&a.z, &b.z, sizeof(a.z)) == 0 && a.base == b.base &&
               std::memcmp(a.x.data(), b.x.data(), sizeof(double) * n) == 0;
    };
    const long long fb0 = g_cfg.fused_batches, hr0 = g_cfg.hang_recoveries;
    Answer a32, a64;
    if (check_p2p) {
        a32 = solve(1, SX_HMAX);
        a64 = solve(1, SX_KMAX);
    }
    const bool went_fused = check_p2p && g_cfg.fused_batches > fb0 && g_cfg.hang_recoveries == hr0;
    const Answer xch = solve(0, 0);
    g_cfg.single_shard = true;  // the reference: one shard of the reference device
    int cur_dev = 0;
    SX_HIP(hipGetDevice(&cur_dev));
    if (ref_dev >= 0) g_cfg.device = ref_dev;
    const Answer one = solve(-1, 0);
    g_cfg.device = save_dev;
    SX_HIP(hipSetDevice(cur_dev));
    g_cfg.single_shard = save_single;
    g_cfg.p2p = save;
    g_cfg.batch = save_batch;
    g_cfg.no_timer = save_nt;
    const int code = !same(xch, one) ? 0 : (went_fused && same(a32, one) && same(a64, one)) ? 2 : 1;
    freeProblem(P);
    free(P);
    return code;
}

// One process, several GPUs (SIMPLEX_GPUS): once per device list and process, selftest_solves
// decides how the list is used: 2 peer-memory fused batches, 1 the per-pivot
// exchange, 0 not at all (every solve on the list's first device).  -1 while the check runs.
int gpus_check(const std::vector<int> &devs) {
    const bool with_p2p = g_cfg.p2p != 0;
    auto &done = with_p2p ? g_cfg.gpus_checked : g_cfg.gpus_checked_xchg;
    auto it = done.find(devs);
    if (it != done.end()) return it->second;
    done[devs] = -1;  // (the check's own engines run the list)
    const int code = selftest_solves((int)devs.size(), devs[0]);
    done[devs] = code;
    if (code == 1 && with_p2p)  // (with peer memory off, 1 is the best a check can return)
        fprintf(stderr, "simplex: peer-memory fused batches disagree with the one-shard answer on these GPUs; "
                        "using the per-pivot exchange\n");
    if (code == 0)
        fprintf(stderr, "simplex: the GPUs of this device list disagree with the one-shard answer; solving on "
                        "device %d alone\n", devs[0]);
    return code;
}
bool gpus_selftest(const std::vector<int> &devs) { return gpus_check(devs) == 2; }

}  // namespace

// ====================================================================== C-ABI
extern "C" {

int simplex_version(void) { return 1; }
void simplex_set_verbose(int on) { g_cfg.verbose = on; }
void simplex_set_sweep_mfma(int mode) { g_cfg.sweep_mfma = mode < 0 ? -1 : (mode ? 1 : 0); }
void simplex_set_batch(int pivots) { g_cfg.batch = pivots > 0 ? std::min(pivots, SX_KMAX) : 0; }
void simplex_set_device(int device) {
    g_cfg.device = device;
    if (device >= 0) SX_HIP(hipSetDevice(device));
}
void simplex_set_virtual_ranks(int world) { g_cfg.virtual_ranks = world > 1 ? world : 1; }
void simplex_set_gpus(const int *devices, int count) {
    g_cfg.gpus.clear();
    for (int i = 0; devices != nullptr && i < count; ++i) g_cfg.gpus.push_back(devices[i]);
}
int simplex_gpus(int *devices, int cap) {
    const std::vector<int> v = shard_devices();
    for (int i = 0; devices != nullptr && i < cap && i < (int)v.size(); ++i) devices[i] = v[(size_t)i];
    return (int)v.size();
}
void simplex_set_force_exchange(int on) { g_cfg.force_exchange = on ? 1 : 0; }
void simplex_set_alias(int on) { g_cfg.alias = on ? 1 : 0; }
void simplex_set_regions(int mode) { g_cfg.regions = mode < 0 ? 1 : mode; }
void simplex_set_mr_single_launch(int on) { g_cfg.mr_single_launch = on ? 1 : 0; }
void simplex_set_compact(int on) { g_cfg.compact = on ? 1 : 0; }
void simplex_set_deactivate(int every) { g_cfg.deact = every > 0 ? every : 0; }
void simplex_set_fused(int mode) { g_cfg.fused = mode < 0 ? -1 : (mode ? 1 : 0); }
void simplex_set_p2p(int mode) { g_cfg.p2p = mode < 0 ? -1 : (mode ? 1 : 0); }
int simplex_p2p_ready(void) {
    const std::vector<int> v = g_cfg.dist ? std::vector<int>() : shard_devices();
    if (v.size() > 1) {  // one process, several GPUs: the self-check of this device list
        auto it = g_cfg.gpus_checked.find(v);
        return it != g_cfg.gpus_checked.end() && it->second == 2 ? 1 : 0;
    }
    return g_cfg.p2p_ready ? 1 : 0;
}
int simplex_multi_gpu_mode(void) {
    const std::vector<int> v = g_cfg.dist ? std::vector<int>() : shard_devices();
    if (v.size() > 1) {
        const auto &done = g_cfg.p2p != 0 ? g_cfg.gpus_checked : g_cfg.gpus_checked_xchg;
        auto it = done.find(v);
        return it == done.end() ? -1 : it->second;
    }
    if (!g_cfg.dist) return -1;
    return g_cfg.single_shard ? 0 : g_cfg.p2p_ready ? 2 : 1;
}
void simplex_last_phase_seconds(double *out) {
    out[0] = g_phase_seconds[0];
    out[1] = g_phase_seconds[1];
}
long long simplex_last_objective_row(double *out, long long cap) {
    const long long n = (long long)g_last_d.size();
    for (long long j = 0; out != nullptr && j < n && j < cap; ++j) out[j] = g_last_d[(size_t)j];
    return n;
}
void simplex_set_update_waves(double waves) { sx_set_update_waves((float)waves); }
void simplex_set_exchange_mode(int mode) { g_cfg.exchange_mode = (mode >= 0 && mode <= 2) ? mode : 0; }
void simplex_set_timer_dir(const char *dir) { g_cfg.timer_dir = dir ? dir : ""; }

void simplex_set_hang_inject(long long batches) { g_cfg.inject_hang = batches >= 0 ? batches : -1; }
void simplex_set_hang_inject_slot(int slot) { g_cfg.inject_slot = slot >= 0 ? slot : -1; }
long long simplex_hang_recoveries(void) { return g_cfg.hang_recoveries; }
long long simplex_fused_batches(void) { return g_cfg.fused_batches; }
void simplex_set_fine_pivot_rows(int mode) { g_cfg.fine_u = mode < 0 ? -1 : mode > 2 ? 1 : mode; }
void simplex_set_replicated_objective(int mode) { g_cfg.repl_obj = mode < 0 ? -1 : (mode ? 1 : 0); }
void simplex_set_check_pivot_rows(int on) { g_cfg.check_u = on ? 1 : 0; }
long long simplex_pivot_row_mismatches(void) { return g_cfg.u_mismatches; }
void simplex_set_blocked(int mode) { g_cfg.blocked = mode < 0 ? -1 : (mode ? 1 : 0); }
void simplex_set_first_batch_id(unsigned int id) { g_cfg.first_batch_id = (id >= 1 && id < SX_BATCH_IDS) ? id : 1; }

void enableBenchmarkMode(void) { g_cfg.benchmark = true; }
void disableBenchmarkMode(void) { g_cfg.benchmark = false; }

int simplex_dist_unique_id_size(void) { return (int)sizeof(ncclUniqueId); }

int simplex_dist_get_unique_id(unsigned char *out) {
    ncclUniqueId id;
    SX_NCCL(ncclGetUniqueId(&id));
    std::memcpy(out, &id, sizeof(id));
    return 0;
}

// The multi-rank fused batch runs over peer memory; before trusting it on this machine, solve
// a small instance with it and with the per-pivot RCCL exchange: it is used only when every
// rank gets bit-identical answers from both.
static void p2p_selftest() {
    g_cfg.p2p_ready = false;
    g_cfg.single_shard = false;
    int code = selftest_solves(g_cfg.world, -1);
    int *dv = nullptr;
    SX_HIP(hipMalloc(reinterpret_cast<void **>(&dv), sizeof(int)));
    SX_HIP(hipMemcpy(dv, &code, sizeof(int), hipMemcpyHostToDevice));
    SX_NCCL(ncclAllReduce(dv, dv, 1, ncclInt, ncclMin, g_cfg.comm, nullptr));
    SX_HIP(hipMemcpy(&code, dv, sizeof(int), hipMemcpyDeviceToHost));
    (void)hipFree(dv);
    g_cfg.p2p_ready = code == 2 && g_cfg.p2p != 0 && g_cfg.world <= SX_MAXW;
    g_cfg.single_shard = code == 0;
    if (code == 1 && g_cfg.p2p != 0 && g_cfg.rank == 0)  // (peer memory off: only the exchange was checked)
        fprintf(stderr, "simplex: peer-memory fused batches disagree with the one-shard answer; using RCCL\n");
    if (code == 0 && g_cfg.rank == 0)
        fprintf(stderr, "simplex: the RCCL exchange disagrees with the one-shard answer; every rank solves alone\n");
}

int simplex_dist_init(int rank, int world, const unsigned char *unique_id, int device) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (device >= 0) {
        g_cfg.device = device;
        SX_HIP(hipSetDevice(device));
    }
    g_cfg.rank = rank;
    g_cfg.world = world;
    if (world > 1 || g_cfg.force_exchange) {
        ncclUniqueId id;
        std::memcpy(&id, unique_id, sizeof(id));
        SX_NCCL(ncclCommInitRank(&g_cfg.comm, world, id, rank));
        g_cfg.dist = true;
        if (world > 1) p2p_selftest();
    }
    return 0;
}

int simplex_dist_finalize(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_cfg.comm) {
        ncclCommDestroy(g_cfg.comm);
        g_cfg.comm = nullptr;
    }
    g_cfg.dist = false;
    g_cfg.world = 1;
    g_cfg.rank = 0;
    return 0;
}

int twoPhaseMethod(problem_t *problem, TYPE *solution, TYPE *optimalValue) {
    return public_status(two_phase(problem, solution, optimalValue, nullptr, nullptr, -1));
}

int twoPhaseMethodEx(problem_t *problem, double *solution, double *optimalValue, int *base_out,
                     long long *pivots_out, long long max_pivots) {
    return two_phase(problem, solution, optimalValue, base_out, pivots_out, max_pivots);
}

// ---------------------------------------------------------------- tabular_t API
// tabular.cu:25-39.  The caller fills the tableau itself, so every one of its 1+n+2m columns is
// stored (no artificial-column aliasing: the caller's artificial columns need not equal the
// slacks) and slack compaction stays off (any column may hold anything): row i occupies
// `rows` doubles at table + i * pitch bytes, exactly as include/tabular.h states.
tabular_t *newTabular(problem_t *problem) {
    Engine *E = new Engine(problem->vars, problem->constraints, /*alias_=*/false);
    tabular_t *t = (tabular_t *)malloc(sizeof(tabular_t));
    t->problem = problem;
    t->cols = problem->constraints;
    t->rows = E->N1;
    t->pitch = E->ld * sizeof(double);
    t->table = E->sh[0].T;
    t->knownTermsVector = E->sh[0].T;
    t->constraintsMatrix = E->sh[0].T + 1;
    t->costsVector = E->sh[0].d;
    g_tabs[t] = E;
    return t;
}

void freeTabular(tabular_t *tabular) {
    auto it = g_tabs.find(tabular);
    if (it != g_tabs.end()) {
        delete it->second;
        g_tabs.erase(it);
    }
    free(tabular);
}

// solve(tabular_t*, int*) (solver.cu:128-149): the caller's base is copied in and out.
int solve(tabular_t *tabular, int *base) {
    auto it = g_tabs.find(tabular);
    if (it == g_tabs.end()) SX_FATAL("solve: unknown tabular");
    Engine *E = it->second;
    // the phase width: 1+n+2m as built, 1+n+m after the caller's `rows -= cols` (phase 2,
    // twoPhaseMethod.cu:288); anything wider than the allocation is refused
    if (tabular->rows < 2 || tabular->rows > E->N1 || tabular->cols != E->m ||
        tabular->pitch != E->ld * sizeof(double))
        SX_FATAL("solve: tabular_t fields do not match its newTabular allocation");
    E->write_base(base);
    long long piv = 0;
    int st = E->run_phase(tabular->rows, -1, &piv);
    E->read_base(base);
    return public_status(st);
}

// tabular.cu:41-98, reference (transposed) orientation
void printTableauToStream(FILE *Stream, tabular_t *tabular, int *base) {
    auto it = g_tabs.find(tabular);
    if (it == g_tabs.end() || tabular->table == nullptr) return;
    Engine *E = it->second;
    const int width = tabular->rows, m = tabular->cols;
    std::vector<double> T((size_t)m * width), d(width);
    E->download(T.data(), width, width, d.data());
    fprintf(Stream, "\n--------------- Tabular --------------\n");
    for (int j = 0; j < width; ++j) {
        for (int i = 0; i < m; ++i) fprintf(Stream, "%.2lf\t", T[(size_t)i * width + j]);
        fprintf(Stream, "\t|\t %.11lf\n", d[j]);
        if (j == 0) fprintf(Stream, "\n");
    }
    fprintf(Stream, "Base\n");
    for (int i = 0; i < m; ++i) fprintf(Stream, "%d\t", base[i]);
}

// ---------------------------------------------------------------- bench sessions
struct simplex_session {
    Engine *E;
    long long total = 0;
    bool started = false;
    std::vector<long long> log_rows;  // per timed launch of the last pivots call
    std::vector<double> log_us;
};

static simplex_session *session_finish(simplex_session *S);

simplex_session *simplex_session_open(problem_t *problem) {
    simplex_session *S = new simplex_session;
    S->E = new Engine(problem->vars, problem->constraints);
    S->E->build_phase1(problem);
    return session_finish(S);
}

simplex_session *simplex_session_open_generated(int n, int m, unsigned int seed, int lo, int hi, int rand_kind) {
    simplex_session *S = new simplex_session;
    S->E = new Engine(n, m);
    S->E->build_phase1_generated(seed, lo, hi, rand_kind);
    return session_finish(S);
}

static simplex_session *session_finish(simplex_session *S) {
    S->E->update_objective(S->E->N1);
    S->E->N = S->E->N1;
    S->E->reset_state(-1);
    S->E->enqueue_enter_partials();
    S->E->sync_all();
    return S;
}

int simplex_session_pivots(simplex_session *S, long long k, int time_updates, simplex_timing_t *out) {
    // k pivots in batches of the configured size, each batch ending with a sweep of the
    // tableau (a call ends with one too, so T is materialised on return).  time_updates =
    // s > 0: bracket every s-th sweep with HIP events and log how many pivots it applied.
    Engine &E = *S->E;
    int K = E.batch_size();
    if (!E.fused_ok(K)) K = std::min(K, SX_HMAX);
    const long long every = time_updates > 0 ? time_updates : 0;
    const long long max_sweeps = (k + K - 1) / K + 1;
    const long long nt = every ? (max_sweeps + every - 1) / every : 0;
    std::vector<hipEvent_t> evs(2 * (size_t)nt);
    for (auto &e : evs) SX_HIP(hipEventCreate(&e));
    std::vector<unsigned> ids((size_t)(nt > 0 ? nt : 1), 0u);
    // (batch_tag, batch_count, swept slack columns) after each timed sweep: the pivots it
    // applied and its width
    int *tag_dev = dalloc<int>((size_t)(nt > 0 ? nt : 1) * 3);
    hipEvent_t w0, w1;
    SX_HIP(hipEventCreate(&w0));
    SX_HIP(hipEventCreate(&w1));
    const long long before = E.read_state().pivots;
    long long nsw = 0, ntimed = 0;
    const bool fused = E.fused_ok(K);
    auto sweep = [&]() {
        const bool timed = every && (nsw % every == 0) && ntimed < nt;
        const unsigned id = E.batch_id;
        // a timed sweep of shard 0 records its batch tag, count and swept slack columns itself
        // (sx_set_sweep_record: no device copies between the kernels of the timed region)
        if (timed) sx_set_sweep_record(tag_dev + 3 * ntimed);
        E.enqueue_sweep(timed ? evs[2 * ntimed] : nullptr, timed ? evs[2 * ntimed + 1] : nullptr, timed);
        sx_set_sweep_record(nullptr);
        if (timed) {
            ids[(size_t)ntimed] = id;
            ++ntimed;
        }
        ++nsw;
    };
    SX_HIP(hipEventRecord(w0, E.s));
    for (long long i = 0; i < k;) {
        if (fused) {
            const int kb = (int)std::min<long long>(K, k - i);
            E.enqueue_batch(kb);
            i += kb;
        } else {
            E.enqueue_pivot();
            ++i;
        }
        if (E.q_host >= K || (fused && E.q_host > 0)) sweep();
    }
    if (E.q_host > 0) sweep();
    E.join();  // (the engine stream's end event follows every device's work)
    SX_HIP(hipEventRecord(w1, E.s));
    SX_HIP(hipEventSynchronize(w1));
    E.sync_all();
    DevState f = E.read_state();
    simplex_timing_t t;
    std::memset(&t, 0, sizeof(t));
    float ms = 0.f;
    SX_HIP(hipEventElapsedTime(&ms, w0, w1));
    t.wall_ms = ms;
    t.pivots = f.pivots - before;
    t.status = f.status;
    t.width = E.N;
    long long rows = 0;
    for (auto &x : E.sh) rows += x.rows;
    t.local_rows = rows;
    t.stored_width = E.cols(E.N).Ns;
    std::vector<int> tags((size_t)(nt > 0 ? nt : 1) * 3, 0);
    SX_HIP(hipMemcpy(tags.data(), tag_dev, sizeof(int) * tags.size(), hipMemcpyDeviceToHost));
    (void)hipFree(tag_dev);
    S->log_rows.clear();
    S->log_us.clear();
    for (long long i = 0; i < ntimed; ++i) {
        // a sweep whose batch selected no pivot (the phase had ended) is a no-op launch
        const int applied = (unsigned)tags[3 * i] == ids[(size_t)i] ? tags[3 * i + 1] : 0;
        if (applied <= 0) continue;
        float us = 0.f;
        SX_HIP(hipEventElapsedTime(&us, evs[2 * i], evs[2 * i + 1]));
        // columns the sweep moved: all stored ones, or 1+n+nact under slack compaction
        const int width = E.compact ? std::min(t.stored_width, 1 + E.n + tags[3 * i + 2]) : t.stored_width;
        t.update_ms += us;
        t.update_launches += 1;
        t.swept_pivots += applied;
        t.swept_bytes += 16.0 * (double)rows * (double)width;
        S->log_rows.push_back(applied);
        S->log_us.push_back(1e3 * (double)us);
    }
    // bytes per timed sweep (their mean, when compaction grows the swept block)
    t.update_bytes = t.update_launches ? t.swept_bytes / (double)t.update_launches
                                       : 16.0 * (double)rows * (double)t.stored_width;
    for (auto &e : evs) (void)hipEventDestroy(e);
    (void)hipEventDestroy(w0);
    (void)hipEventDestroy(w1);
    S->total = f.pivots;
    if (!E.ipc) E.gather_d();  // (outside the timed region: the whole objective row on every shard)
    E.sync_all();
    if (out) *out = t;
    return f.status;
}

double simplex_session_objective(simplex_session *S) { return S->E->read_d0(); }

long long simplex_session_tableau(simplex_session *S, double *T, long long ld, double *d, int *base) {
    Engine &E = *S->E;
    if (E.rccl || ld < E.N) return -1;
    E.download(T, (size_t)ld, E.N, d);
    E.read_base(base);
    return E.N;
}

long long simplex_session_active_slacks(simplex_session *S) { return S->E->active_slacks(); }
long long simplex_session_total_pivots(simplex_session *S) { return S->E->read_state().pivots; }
int simplex_session_batch(simplex_session *S) {
    const int K = S->E->batch_size();
    return S->E->fused_ok(K) ? K : std::min(K, SX_HMAX);
}

int simplex_session_stamps(simplex_session *S, int k, unsigned long long *out) {
    return simplex_session_block_stamps(S, k, out, nullptr, 0) < 0 ? -1 : 0;
}

int simplex_session_block_stamps(simplex_session *S, int k, unsigned long long *out, unsigned long long *blk,
                                 long long cap) {
    // one fused batch of k pivots with in-kernel timestamps (diagnostic); out[k][8], and
    // blk[k][blocks][4] when it holds cap >= k * blocks * 4 entries; returns the blocks
    Engine &E = *S->E;
    if (k < 1 || k > SX_KMAX || !E.fused_ok(k) || E.sh.size() != 1) return -1;
    const size_t nb = (size_t)((E.sh[0].rows + SX_TILE - 1) / SX_TILE) + (size_t)((E.N - 1 + SX_TILE - 1) / SX_TILE);
    const size_t total = (size_t)k * 8 + (size_t)k * nb * 4;
    unsigned long long *dev = dalloc<unsigned long long>(total);
    SX_HIP(hipMemsetAsync(dev, 0, sizeof(unsigned long long) * total, E.s));
    E.stamps = dev;
    E.enqueue_batch(k);
    E.stamps = nullptr;
    E.enqueue_sweep();
    if (!E.ipc) E.gather_d();
    E.sync_all();
    SX_HIP(hipMemcpyAsync(out, dev, sizeof(unsigned long long) * k * 8, hipMemcpyDeviceToHost, E.s));
    if (blk && cap >= (long long)((size_t)k * nb * 4))
        SX_HIP(hipMemcpyAsync(blk, dev + (size_t)k * 8, sizeof(unsigned long long) * k * nb * 4, hipMemcpyDeviceToHost,
                              E.s));
    SX_HIP(hipStreamSynchronize(E.s));
    (void)hipFree(dev);
    return (int)nb;
}

long long simplex_session_launch_log(simplex_session *S, long long *rows, double *update_us, long long cap) {
    const long long n = (long long)S->log_rows.size();
    for (long long i = 0; i < n && i < cap; ++i) {
        if (rows) rows[i] = S->log_rows[(size_t)i];
        if (update_us) update_us[i] = S->log_us[(size_t)i];
    }
    return n;
}

void simplex_session_close(simplex_session *S) {
    if (!S) return;
    delete S->E;
    delete S;
}

// ---- multi-process peer-memory test mode (no RCCL): see simplex_hip.h
int simplex_ipc_handles_size(void) { return (int)Engine::kHandles; }

simplex_session *simplex_ipc_session_open(int n, int m, int rank, int world, const double *T_rows, long long ld_host,
                                          const double *d, const int *base, unsigned char *handles_out) {
    if (world < 2 || world > SX_MAXW || rank < 0 || rank >= world) return nullptr;
    const long long N1 = 1 + (long long)n + 2LL * m;
    g_cfg.ipc_rank = rank;
    g_cfg.ipc_world = world;
    simplex_session *S = new simplex_session;
    // probe the shard's row range with a throw-away shape first: aliasing needs this rank's rows
    // to satisfy the artificial == slack invariant (true for any fresh phase-1 state)
    const int W = world;
    const int rpr = (int)round_up((size_t)((m + W - 1) / W), SX_TILE);
    const int row0 = rank * rpr, rows = std::max(0, std::min(rpr, m - row0));
    // (every rank must store the same columns: a rank without rows follows the invariant)
    const bool alias = rows == 0 || artificial_equals_slack(T_rows, rows, N1, ld_host, n, m);
    S->E = new Engine(n, m, alias);
    g_cfg.ipc_rank = -1;
    g_cfg.ipc_world = 0;
    Engine &E = *S->E;
    E.upload(T_rows, (size_t)ld_host, (int)N1, d, base, /*local_rows=*/true);
    E.N = E.N1;
    E.reset_state(-1);
    E.enqueue_enter_partials();
    E.sync_all();
    if (!E.export_handles(handles_out)) {
        simplex_session_close(S);
        return nullptr;
    }
    return S;
}

int simplex_ipc_session_connect(simplex_session *S, const unsigned char *all_handles) {
    Engine &E = *S->E;
    if (!E.ipc || !E.map_peers(all_handles, E.sh[0].rank)) return -1;
    E.p2p = true;
    return E.fused_ok(E.batch_size()) ? 0 : -2;
}

int simplex_session_sync_d(simplex_session *S) {
    Engine &E = *S->E;
    if (!E.ipc) return -1;
    E.publish_d_ipc();
    return 0;
}

long long simplex_session_rows(simplex_session *S, double *T_rows, long long ld_host, double *d, int *base) {
    Engine &E = *S->E;
    if (ld_host < E.N) return -1;
    // IPC ranks keep only their own slice of d current between fused batches: the whole row
    // exists only after simplex_session_sync_d (every process) -- refuse a stale read
    if (E.ipc && E.d_split) return -2;
    E.download(T_rows, (size_t)ld_host, E.N, d, /*local_rows=*/true);
    E.read_base(base);
    return E.sh[0].rows;
}

// ---------------------------------------------------------------- synthetic sweep bench
// SURVEY.md §8d config 3': the production sweep kernel (k_sweep) on a synthetic rows x cols
// fp64 matrix -- entries uniform in [lo, hi] drawn as generateRandomProblem draws A
// (problem.cu:49-126, seed's third CRT draw) -- with `pivots` random pending pivots: row
// factors in [-1, 1), pivot rows in [lo, hi], distinct leaving rows (their entries take the
// divide path of solver.cu:40-43).  The matrix is swept `warmup` + `iters` times in place;
// the `iters` timed sweeps are bracketed by HIP events on the sweep's stream.  Returns the
// average microseconds per sweep; *bytes = 16 * rows * cols (each element read and written
// once, SURVEY.md §8d's 16 (m+1) N figure for this matrix).
double simplex_bench_sweep(int rows, int cols, unsigned int seed, int lo, int hi, int pivots, int warmup, int iters,
                           double *bytes) {
    if (rows <= 0 || cols <= 1 || pivots < 1 || pivots > SX_KMAX || iters < 1 || rows < pivots) return -1.0;
    const size_t ld = round_up((size_t)cols, 16);
    hipStream_t s;
    SX_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t sd[3];
    sx_crt_seeds(seed, 0, sd);
    TLay btl;  // one region, the engine's storage (row-major, or 4x4 blocks in whole 16-row strips)
    btl.ldA = ld;
    btl.jB = cols;
    btl.blk = use_blocked() ? 1 : 0;
    const size_t rows_alloc = btl.blk ? round_up((size_t)rows, 16) : (size_t)rows;
    double *T = dalloc<double>(rows_alloc * btl.ldA);
    double *U = dalloc<double>((size_t)SX_KMAX * ld);
    double *F = dalloc<double>(round_up((size_t)rows, 16) * SX_KMAX);
    PivRec *recs = dalloc<PivRec>(SX_KMAX);
    unsigned long long *PM = dalloc<unsigned long long>(rows);
    unsigned long long *PM2 = dalloc<unsigned long long>(rows);
    DevState *st = dalloc<DevState>(1);
    SX_HIP(hipMemsetAsync(T, 0, sizeof(double) * rows_alloc * btl.ldA, s));
    // column 0 = b (first CRT seed), columns 1.. = A's rows (third), as generateRandomProblem
    double *b_dev = dalloc<double>(rows);
    sx_launch_gen_vector(sd[0], 0, rows, lo, hi, b_dev, s);
    sx_launch_gen_rows(sd[2], cols - 1, rows, 0, rows, lo, hi, T, btl, nullptr, s);
    sx_launch_rows_in(T, btl, 0, rows, 1, 0, b_dev, 1, s);
    SX_HIP(hipStreamSynchronize(s));
    (void)hipFree(b_dev);
    SX_HIP(hipMemsetAsync(U, 0, sizeof(double) * SX_KMAX * ld, s));
    for (int k = 0; k < pivots; ++k) sx_launch_gen_vector(sd[1] + 7919u * (unsigned)k, 0, cols, lo, hi, U + k * ld, s);
    sx_launch_gen_vector(sd[1] ^ 0x9e3779b9u, 0, (int)(round_up((size_t)rows, 16) * SX_KMAX), -1, 1, F, s);
    const unsigned B = 1;
    std::vector<PivRec> rc(SX_KMAX);
    std::vector<unsigned long long> pm((size_t)rows, 0ull), pm2((size_t)rows, 0ull);
    // the leaving rows: distinct pseudo-random rows (a fixed LCG of the seed), as the pivot loop's
    // are -- evenly spaced ones (every rows/pivots-th row, rounds 1-4) put every leaving row of a
    // 4096-row sweep into the strips of 2 of its 16 row slots
    std::vector<int> lrow;
    {
        std::vector<unsigned char> used((size_t)rows, 0);
        unsigned long long x = 0x9e3779b97f4a7c15ull ^ seed;
        while ((int)lrow.size() < SX_KMAX) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            const int r = (int)((x >> 33) % (unsigned long long)rows);
            if (used[(size_t)r] && (int)lrow.size() < rows) continue;
            used[(size_t)r] = 1;
            lrow.push_back(r);
        }
    }
    for (int k = 0; k < SX_KMAX; ++k) {
        rc[k].r = lrow[(size_t)k];
        rc[k].e = k;
        rc[k].p = 1.0 + (double)(k % 97);
        if (k < pivots && k < SX_HMAX) pm[(size_t)rc[k].r] = ((unsigned long long)B << 32) | (1ull << k);
        if (k < pivots && k >= SX_HMAX) pm2[(size_t)rc[k].r] = ((unsigned long long)B << 32) | (1ull << (k - SX_HMAX));
    }
    SX_HIP(hipMemcpyAsync(recs, rc.data(), sizeof(PivRec) * SX_KMAX, hipMemcpyHostToDevice, s));
    SX_HIP(hipMemcpyAsync(PM, pm.data(), sizeof(unsigned long long) * rows, hipMemcpyHostToDevice, s));
    SX_HIP(hipMemcpyAsync(PM2, pm2.data(), sizeof(unsigned long long) * rows, hipMemcpyHostToDevice, s));
    DevState init;
    std::memset(&init, 0, sizeof(init));
    init.status = SX_NOT_ENDED;
    init.batch_tag = B;
    init.batch_count = pivots;
    SX_HIP(hipMemcpyAsync(st, &init, sizeof(init), hipMemcpyHostToDevice, s));
    Pending pd;
    pd.U = U;
    pd.F = F;
    pd.recs = recs;
    pd.PM = PM;
    pd.PM2 = PM2;
    pd.batch = B;
    pd.q = pivots;
    SweepCfg cfg;
    cfg.batch = pivots;
    cfg.mfma = pivots > SX_HMAX ? 1 : (g_cfg.sweep_mfma >= 0 ? g_cfg.sweep_mfma : 1);
    long long sweeps = 0;
    auto one = [&]() { sx_launch_sweep(T, rows, 0, ld, btl, cols, nullptr, 0, pd, st, (int)(sweeps & 1), cfg, s); };
    for (int w = 0; w < warmup; ++w, ++sweeps) one();
    hipEvent_t e0, e1;
    SX_HIP(hipEventCreate(&e0));
    SX_HIP(hipEventCreate(&e1));
    SX_HIP(hipEventRecord(e0, s));
    for (int it = 0; it < iters; ++it, ++sweeps) one();
    SX_HIP(hipEventRecord(e1, s));
    SX_HIP(hipEventSynchronize(e1));
    float ms = 0.f;
    SX_HIP(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    for (void *p : {(void *)T, (void *)U, (void *)F, (void *)recs, (void *)PM, (void *)PM2, (void *)st}) (void)hipFree(p);
    (void)hipStreamDestroy(s);
    if (bytes) *bytes = 16.0 * (double)rows * (double)cols;
    return 1e3 * (double)ms / (double)iters;
}

// ---------------------------------------------------------------- parity hooks
long long simplex_dev_argmin(const double *v, long long L, double *vmin) {
    hipStream_t s;
    SX_HIP(hipStreamCreate(&s));
    double *dv = dalloc<double>(L > 0 ? L : 1);
    TilePart *parts = dalloc<TilePart>(SX_TILE);
    int *di = dalloc<int>(1);
    double *dvm = dalloc<double>(1);
    if (L > 0) SX_HIP(hipMemcpyAsync(dv, v, sizeof(double) * L, hipMemcpyHostToDevice, s));
    sx_launch_argmin_vector(dv, L, parts, di, dvm, s);
    int idx = -1;
    double mv = 0.0;
    SX_HIP(hipMemcpyAsync(&idx, di, sizeof(int), hipMemcpyDeviceToHost, s));
    SX_HIP(hipMemcpyAsync(&mv, dvm, sizeof(double), hipMemcpyDeviceToHost, s));
    SX_HIP(hipStreamSynchronize(s));
    (void)hipFree(dv);
    (void)hipFree(parts);
    (void)hipFree(di);
    (void)hipFree(dvm);
    (void)hipStreamDestroy(s);
    if (vmin) *vmin = mv;
    return idx;
}

int simplex_dev_pivots(double *T, long long m, long long N, long long ld, double *d, int *base, long long k,
                       long long *done) {
    // a scratch engine sized for width N: n + 2m + 1 >= N is all it needs; aliased storage
    // only when the caller's tableau satisfies the invariant
    Engine E((int)(N - 1 - 2 * m) > 0 ? (int)(N - 1 - 2 * m) : 0, (int)m, artificial_equals_slack(T, m, N, ld));
    if ((long long)E.cols((int)N).Ns > (long long)E.ld) SX_FATAL("simplex_dev_pivots: width exceeds engine stride");
    E.upload(T, (size_t)ld, (int)N, d, base);
    long long piv = 0;
    const int st = E.run_phase((int)N, k, &piv);
    E.download(T, (size_t)ld, (int)N, d);
    E.read_base(base);
    if (done) *done = piv;
    return st == SX_PIVOT_CAP ? SIMPLEX_NOT_ENDED : st;
}

int simplex_dev_update_objective(const double *T, long long m, long long N, long long ld, const int *base,
                                 double *d) {
    Engine E((int)(N - 1 - 2 * m) > 0 ? (int)(N - 1 - 2 * m) : 0, (int)m, artificial_equals_slack(T, m, N, ld));
    if ((long long)E.cols((int)N).Ns > (long long)E.ld) SX_FATAL("simplex_dev_update_objective: width exceeds engine stride");
    E.upload(T, (size_t)ld, (int)N, d, base);
    E.update_objective((int)N);
    SX_HIP(hipStreamSynchronize(E.s));
    SX_HIP(hipMemcpy(d, E.sh[0].d, sizeof(double) * N, hipMemcpyDeviceToHost));
    return 0;
}

problem_t *sx_malloc_problem(int n, int m);

problem_t *simplex_generate_problem_device(int n, int m, unsigned int seed, int lo, int hi, int rand_kind) {
    problem_t *p = sx_malloc_problem(n, m);
    uint32_t sd[3];
    sx_crt_seeds(seed, rand_kind, sd);
    hipStream_t s;
    SX_HIP(hipStreamCreate(&s));
    double *A = dalloc<double>((size_t)n * m), *b = dalloc<double>(m), *c = dalloc<double>(n);
    sx_launch_gen_vector(sd[0], 0, m, lo, hi, b, s);
    sx_launch_gen_vector(sd[1], 0, n, lo, hi, c, s);
    sx_launch_gen_rows(sd[2], n, m, 0, m, lo, hi, nullptr, TLay(), A, s);
    if (n > 0 && m > 0)
        SX_HIP(hipMemcpyAsync(p->constraintsMatrix, A, sizeof(double) * (size_t)n * m, hipMemcpyDeviceToHost, s));
    if (m > 0) SX_HIP(hipMemcpyAsync(p->knownTermsVector, b, sizeof(double) * m, hipMemcpyDeviceToHost, s));
    if (n > 0) SX_HIP(hipMemcpyAsync(p->objectiveFunction, c, sizeof(double) * n, hipMemcpyDeviceToHost, s));
    SX_HIP(hipStreamSynchronize(s));
    (void)hipFree(A);
    (void)hipFree(b);
    (void)hipFree(c);
    (void)hipStreamDestroy(s);
    return p;
}

int simplex_dev_build_phase1_generated(int n, int m, unsigned int seed, int lo, int hi, double *T, long long ld,
                                       double *d, int *base) {
    Engine E(n, m);
    E.build_phase1_generated(seed, lo, hi, 0);
    E.download(T, (size_t)ld, E.N1, d);
    E.read_base(base);
    return 0;
}

int simplex_dev_build_phase1(problem_t *problem, double *T, long long ld, double *d, int *base) {
    Engine E(problem->vars, problem->constraints);
    E.build_phase1(problem);
    E.download(T, (size_t)ld, E.N1, d);
    E.read_base(base);
    return 0;
}

}  // extern "C"
