"""Python mirror of the reference host API, over the C-ABI of libsimplex_hip.so.

Names, argument meaning and status codes follow the reference headers:
  problem.h (readProblemFromFile, readRandomProblemFromFile, generateRandomProblem,
  printProblemToStream, freeProblem), twoPhaseMethod.h (twoPhaseMethod, FEASIBLE ...).
The compute always runs in the HIP library on the GPU; this module only marshals arrays.
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib

FEASIBLE = 0
INFEASIBLE = -1
UNBOUNDED = -2
DEGENERATE = -3
NOT_ENDED = -10
PIVOT_CAP = -11
NUMERIC_FAIL = -12
HANG = -13

STATUS_NAMES = {FEASIBLE: "FEASIBLE", INFEASIBLE: "INFEASIBLE", UNBOUNDED: "UNBOUNDED",
                DEGENERATE: "DEGENERATE", NOT_ENDED: "NOT_ENDED", PIVOT_CAP: "PIVOT_CAP",
                NUMERIC_FAIL: "NUMERIC_FAIL", HANG: "HANG"}

RAND_MSVC = 0
RAND_GLIBC = 1

_libc = ctypes.CDLL(None)
_libc.fopen.restype = ctypes.c_void_p
_libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
_libc.fclose.argtypes = [ctypes.c_void_p]
_libc.fflush.argtypes = [ctypes.c_void_p]


def _dp(a):
    return a.ctypes.data_as(_lib.c_double_p)


def _ip(a):
    return a.ctypes.data_as(_lib.c_int_p)


class Problem:
    """Owns a problem_t* allocated by the library (A column-major, problem.h:10-26)."""

    def __init__(self, ptr):
        if not ptr:
            raise ValueError("null problem_t")
        self._ptr = ptr

    @property
    def ptr(self):
        return self._ptr

    @property
    def n(self):
        return self._ptr.contents.vars

    @property
    def m(self):
        return self._ptr.contents.constraints

    def arrays(self):
        """Copies of (A as an m x n array, b, c)."""
        p = self._ptr.contents
        n, m = p.vars, p.constraints
        A_cm = np.ctypeslib.as_array(p.constraintsMatrix, shape=(n * m,)).copy() if n * m else np.zeros(0)
        A = A_cm.reshape(n, m).T.copy() if n * m else np.zeros((m, n))
        b = np.ctypeslib.as_array(p.knownTermsVector, shape=(m,)).copy() if m else np.zeros(0)
        c = np.ctypeslib.as_array(p.objectiveFunction, shape=(n,)).copy() if n else np.zeros(0)
        return A, b, c

    @classmethod
    def from_arrays(cls, A, b, c):
        A = np.asarray(A, dtype=np.float64)
        m, n = A.shape
        A_cm = np.ascontiguousarray(A.T).reshape(-1)
        b = np.ascontiguousarray(b, dtype=np.float64)
        c = np.ascontiguousarray(c, dtype=np.float64)
        lib = _lib.load()
        return cls(lib.simplex_problem_from_arrays(n, m, _dp(A_cm), _dp(b), _dp(c)))

    def close(self):
        if self._ptr:
            _lib.load().simplex_free_problem_struct(self._ptr)
            self._ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def generateRandomProblem(nVars, nConstraints, seed, minGenerator=-100, maxGenerator=100, rand_kind=RAND_MSVC):
    """problem.cu:49-126 (defaults of problem.h:54)."""
    lib = _lib.load()
    return Problem(lib.simplex_generate_problem_ex(nVars, nConstraints, seed & 0xFFFFFFFF, minGenerator,
                                                   maxGenerator, rand_kind))


def generateRandomProblemDevice(nVars, nConstraints, seed, minGenerator=-100, maxGenerator=100,
                                rand_kind=RAND_MSVC):
    """generateRandomProblem computed on the GPU (bit-identical to the host generator)."""
    lib = _lib.load()
    return Problem(lib.simplex_generate_problem_device(nVars, nConstraints, seed & 0xFFFFFFFF, minGenerator,
                                                       maxGenerator, rand_kind))


def _with_file(path, mode, fn):
    f = _libc.fopen(str(path).encode(), mode.encode())
    if not f:
        raise OSError(f"Cannot open file! ({path})")
    try:
        return fn(f)
    finally:
        _libc.fclose(f)


def readProblemFromFile(path):
    """problem.cu:20-47."""
    lib = _lib.load()
    return Problem(_with_file(path, "r", lib.readProblemFromFile))


def readRandomProblemFromFile(path):
    """problem.cu:128-139 ("n m seed min max")."""
    lib = _lib.load()
    return Problem(_with_file(path, "r", lib.readRandomProblemFromFile))


def printProblemToStream(problem, path):
    """problem.cu:141-181, written to `path`."""
    lib = _lib.load()
    _with_file(path, "w", lambda f: lib.printProblemToStream(f, problem.ptr))


@dataclass
class Result:
    status: int
    solution: np.ndarray
    optimal_value: float
    base: np.ndarray
    pivots: tuple

    @property
    def status_name(self):
        return STATUS_NAMES.get(self.status, str(self.status))


def twoPhaseMethod(problem):
    """twoPhaseMethod.h:19 -> (status, solution, optimalValue)."""
    lib = _lib.load()
    x = np.zeros(max(problem.n, 1))
    opt = ctypes.c_double(0.0)
    st = lib.twoPhaseMethod(problem.ptr, _dp(x), ctypes.byref(opt))
    return st, x[:problem.n], opt.value


def twoPhaseMethodEx(problem, max_pivots=-1):
    """twoPhaseMethod + final basis and per-phase pivot counts (simplex_hip.h)."""
    lib = _lib.load()
    x = np.zeros(max(problem.n, 1))
    base = np.zeros(max(problem.m, 1), dtype=np.int32)
    piv = (ctypes.c_longlong * 2)()
    opt = ctypes.c_double(0.0)
    st = lib.twoPhaseMethodEx(problem.ptr, _dp(x), ctypes.byref(opt), _ip(base), piv, max_pivots)
    return Result(st, x[:problem.n], opt.value, base[:problem.m], (piv[0], piv[1]))


def last_objective_row():
    """The last twoPhaseMethod call's final objective row (simplex_last_objective_row)."""
    lib = _lib.load()
    n = lib.simplex_last_objective_row(None, 0)
    d = np.zeros(max(n, 1))
    lib.simplex_last_objective_row(_dp(d), n)
    return d[:n]


class Session:
    """A resident phase-1 tableau on this process's GPU shard, for timed pivots."""

    def __init__(self, problem=None, generated=None):
        """problem: a Problem; or generated=(n, m, seed, lo, hi) to synthesise the tableau in HBM."""
        self._lib = _lib.load()
        if generated is not None:
            n, m, seed, lo, hi = generated
            self._h = self._lib.simplex_session_open_generated(n, m, seed & 0xFFFFFFFF, lo, hi, RAND_MSVC)
        else:
            self._h = self._lib.simplex_session_open(problem.ptr)
        if not self._h:
            raise RuntimeError("simplex_session_open failed")

    def pivots(self, k, time_updates=0):
        """k pivots (ending with a sweep, so the tableau is materialised); time_updates = s > 0
        times every s-th tableau sweep with HIP events."""
        t = _lib.TimingT()
        self._lib.simplex_session_pivots(self._h, k, int(time_updates), ctypes.byref(t))
        return t

    def launch_log(self):
        """(pivots applied, sweep microseconds) per timed sweep of the last pivots() call."""
        n = self._lib.simplex_session_launch_log(self._h, None, None, 0)
        rows = np.zeros(max(n, 1), dtype=np.int64)
        us = np.zeros(max(n, 1), dtype=np.float64)
        self._lib.simplex_session_launch_log(self._h, rows.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)),
                                             _dp(us), n)
        return rows[:n], us[:n]

    def stamps(self, k):
        """Diagnostic: one fused batch of k pivots with in-kernel timestamps, (k, 8) uint64 in
        10-ns ticks (see simplex_session_stamps); None when the fused path is not in use."""
        out = np.zeros((k, 8), dtype=np.uint64)
        rc = self._lib.simplex_session_stamps(self._h, k, out.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)))
        return out if rc == 0 else None

    def block_stamps(self, k, blocks):
        """Diagnostic: stamps(k) plus every block's own, (k, blocks, 4) uint64 (see
        simplex_session_block_stamps); (None, None) when the fused path is not in use."""
        out = np.zeros((k, 8), dtype=np.uint64)
        blk = np.zeros((k, blocks, 4), dtype=np.uint64)
        P = ctypes.POINTER(ctypes.c_ulonglong)
        rc = self._lib.simplex_session_block_stamps(self._h, k, out.ctypes.data_as(P), blk.ctypes.data_as(P), blk.size)
        if rc < 0:
            return None, None
        if rc != blocks:
            raise RuntimeError(f"simplex_session_block_stamps: {rc} blocks, expected {blocks}")
        return out, blk

    def objective(self):
        return self._lib.simplex_session_objective(self._h)

    def tableau(self, m, width):
        """(T, d, base): the resident tableau in logical column order (rows on this process)."""
        T = np.zeros((m, width), dtype=np.float64)
        d = np.zeros(width, dtype=np.float64)
        base = np.zeros(m, dtype=np.int32)
        w = self._lib.simplex_session_tableau(self._h, _dp(T), width, _dp(d), _ip(base))
        if w != width:
            raise RuntimeError(f"simplex_session_tableau: width {w}, expected {width}")
        return T, d, base

    def objective_row_and_basis(self, m, width):
        """(d, base) without the tableau (simplex_session_tableau with T null)."""
        d = np.zeros(width, dtype=np.float64)
        base = np.zeros(m, dtype=np.int32)
        w = self._lib.simplex_session_tableau(self._h, None, width, _dp(d), _ip(base))
        if w != width:
            raise RuntimeError(f"simplex_session_tableau: width {w}, expected {width}")
        return d, base

    def active_slacks(self):
        """Slack columns the sweeps move (m without slack compaction)."""
        return self._lib.simplex_session_active_slacks(self._h)

    def total_pivots(self):
        return self._lib.simplex_session_total_pivots(self._h)

    def batch(self):
        """Pivots per batch (and per sweep) of pivots() on this session."""
        return self._lib.simplex_session_batch(self._h)

    def close(self):
        if self._h:
            self._lib.simplex_session_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def bench_sweep(rows, cols, seed, lo=1, hi=100, pivots=32, warmup=3, iters=20):
    """SURVEY.md §8d config 3': the sweep kernel on a synthetic rows x cols matrix;
    returns (average microseconds per sweep, algorithmic bytes per sweep)."""
    b = ctypes.c_double(0.0)
    us = _lib.load().simplex_bench_sweep(rows, cols, seed & 0xFFFFFFFF, lo, hi, pivots, warmup, iters,
                                         ctypes.byref(b))
    if us < 0:
        raise ValueError("simplex_bench_sweep: bad arguments")
    return us, b.value


# ---- kernel-level parity hooks ----
def dev_argmin(v):
    lib = _lib.load()
    v = np.ascontiguousarray(v, dtype=np.float64)
    vm = ctypes.c_double(0.0)
    idx = lib.simplex_dev_argmin(_dp(v), len(v), ctypes.byref(vm))
    return int(idx), vm.value


def dev_pivots(T, d, base, k):
    """k pivots on the device; T (m x ld, width len(d)), d, base updated in place."""
    lib = _lib.load()
    assert T.dtype == np.float64 and T.flags.c_contiguous and d.flags.c_contiguous
    assert base.dtype == np.int32
    m, ld = T.shape
    done = ctypes.c_longlong(0)
    st = lib.simplex_dev_pivots(_dp(T), m, len(d), ld, _dp(d), _ip(base), k, ctypes.byref(done))
    return st, done.value


def dev_update_objective(T, d, base):
    lib = _lib.load()
    m, ld = T.shape
    return lib.simplex_dev_update_objective(_dp(T), m, len(d), ld, _ip(base), _dp(d))


def dev_build_phase1(problem):
    lib = _lib.load()
    n, m = problem.n, problem.m
    N1 = 1 + n + 2 * m
    T = np.zeros((m, N1))
    d = np.zeros(N1)
    base = np.zeros(max(m, 1), dtype=np.int32)
    lib.simplex_dev_build_phase1(problem.ptr, _dp(T), N1, _dp(d), _ip(base))
    return T, d, base[:m]


def dev_build_phase1_generated(n, m, seed, lo, hi):
    lib = _lib.load()
    N1 = 1 + n + 2 * m
    T = np.zeros((m, N1))
    d = np.zeros(N1)
    base = np.zeros(max(m, 1), dtype=np.int32)
    lib.simplex_dev_build_phase1_generated(n, m, seed & 0xFFFFFFFF, lo, hi, _dp(T), N1, _dp(d), _ip(base))
    return T, d, base[:m]


def set_virtual_ranks(w):
    _lib.load().simplex_set_virtual_ranks(int(w))


def set_gpus(devices):
    """One process, several GPUs (simplex_set_gpus): one row-block shard per listed device
    (None or [] = the SIMPLEX_GPUS environment variable decides)."""
    devs = list(devices or [])
    arr = (ctypes.c_int * max(len(devs), 1))(*devs)
    _lib.load().simplex_set_gpus(arr, len(devs))


def gpus():
    """The device list in effect (simplex_set_gpus, else SIMPLEX_GPUS); [] = one shard."""
    lib = _lib.load()
    n = lib.simplex_gpus(None, 0)
    arr = (ctypes.c_int * max(n, 1))()
    lib.simplex_gpus(arr, n)
    return list(arr[:n])


def set_force_exchange(on):
    _lib.load().simplex_set_force_exchange(1 if on else 0)


def set_exchange_mode(mode):
    _lib.load().simplex_set_exchange_mode(int(mode))


def set_alias(on):
    _lib.load().simplex_set_alias(1 if on else 0)


def set_compact(on):
    """Slack compaction (default on): sweeps skip slack columns no pivot has touched."""
    _lib.load().simplex_set_compact(1 if on else 0)


DEACTIVATE_EVERY = 8  # the engine's default


def set_deactivate(every):
    """With slack compaction on one shard: every `every` sweeps (default 8; 0 off) the swept slack
    columns whose slack is basic (exact unit vectors) leave the swept block."""
    _lib.load().simplex_set_deactivate(int(every))


def set_fused(mode):
    """-1 auto (one launch per batch of pivots on a single shard), 0 two launches per pivot."""
    _lib.load().simplex_set_fused(int(mode))


def set_p2p(mode):
    """Several shards: fused batches exchanging over peer memory (-1 auto, 0 off, 1 force)."""
    _lib.load().simplex_set_p2p(int(mode))


def p2p_ready():
    """True when the peer-memory path passed the multi-GPU start-up self-check."""
    return bool(_lib.load().simplex_p2p_ready())


def set_update_waves(w):
    """Blocks of the tableau sweep as a multiple of the device's resident capacity (<= 0: default)."""
    _lib.load().simplex_set_update_waves(float(w))


def set_blocked(mode):
    """New engines' tableau storage: -1 default (the blocked layout unless SIMPLEX_BLOCKED=0), 1 the
    blocked layout (4x4 blocks in 16-row strips), 0 row-major."""
    _lib.load().simplex_set_blocked(int(mode))


def set_fine_pivot_rows(mode):
    """Pending pivot rows U in fine-grained memory: -1 default (when shards sit on different
    devices), 1 always, 0 never."""
    _lib.load().simplex_set_fine_pivot_rows(int(mode))


def set_replicated_objective(mode):
    """Multi-rank fused batches with every rank running every objective tile (one cross-rank hop
    per pivot): -1 default (when shards sit on different devices), 1 always (when
    the grid fits), 0 never."""
    _lib.load().simplex_set_replicated_objective(int(mode))


def set_regions(mode):
    """New engines' tableau layout: 0 plain rows, 1 auto two-region layout (default), >= 2 region A
    forced to that many slack positions (test hook)."""
    _lib.load().simplex_set_regions(int(mode))


def set_mr_single_launch(on):
    """Virtual shards with the peer-memory batch: all ranks' batches in one launch (default) or one
    launch per rank on its own stream."""
    _lib.load().simplex_set_mr_single_launch(1 if on else 0)


def set_verbose(on):
    _lib.load().simplex_set_verbose(1 if on else 0)


def set_sweep_mfma(mode):
    """The tableau sweep on the matrix cores (1), the vector sweep (0) or auto (-1)."""
    _lib.load().simplex_set_sweep_mfma(int(mode))


def set_batch(p):
    """Pivots per tableau sweep (1..64; <= 0: auto -- 64 when the tableau has >= 4096 rows, else 32).
    Batches above 32 run only in the fused batches (one shard's and the peer-memory multi-rank
    one); the per-pivot path caps them at 32 (simplex_hip.h simplex_set_batch)."""
    _lib.load().simplex_set_batch(int(p))
