"""ctypes wrapper of the CPU oracle (liboracle.so).  TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker / timed CPU baseline -- never from the product package.  See oracle.h.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)
_lp = ctypes.POINTER(ctypes.c_int64)
_lib = None

FEASIBLE, INFEASIBLE, UNBOUNDED, DEGENERATE, NOT_ENDED, PIVOT_CAP = 0, -1, -2, -3, -10, -11


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    lib = ctypes.CDLL(LIB_PATH)
    i64 = ctypes.c_int64
    sig = {
        "orc_crt_rand": (None, [ctypes.c_uint, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint32)]),
        "orc_xorwow_draws": (None, [ctypes.c_uint64, ctypes.c_uint64, i64, ctypes.POINTER(ctypes.c_uint32)]),
        "orc_generate_problem": (None, [ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_int, _dp, _dp, _dp]),
        "orc_argmin": (i64, [_dp, i64, _dp]),
        "orc_argmin_tile": (None, [_dp, i64, i64, _dp, _lp]),
        "orc_argmin_pass2": (i64, [_dp, _lp, i64, _dp]),
        "orc_build_phase1": (None, [ctypes.c_int, ctypes.c_int, _dp, _dp, _dp, i64, _dp, _ip]),
        "orc_gemv_partials": (None, [_dp, i64, i64, i64, _dp, _dp]),
        "orc_gemv_apply": (None, [_dp, i64, _dp, i64]),
        "orc_update_objective": (None, [_dp, i64, i64, i64, _ip, _dp]),
        "orc_ratio": (ctypes.c_double, [ctypes.c_double, ctypes.c_double]),
        "orc_apply_update": (None, [_dp, i64, i64, i64, _dp, _dp, _dp, i64, ctypes.c_double, ctypes.c_double]),
        "orc_pivot": (ctypes.c_int, [_dp, i64, i64, i64, _dp, _ip, _lp, _lp]),
        "orc_solve": (ctypes.c_int, [_dp, i64, i64, i64, _dp, _ip, i64, _lp]),
        "orc_two_phase": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _dp, _dp, _dp, i64, _dp, _dp, _ip, _lp, _dp]),
        "orc_last_objective_row": (i64, [_dp, i64]),
        "orc_set_threads": (None, [ctypes.c_int]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def p(a):
    return a.ctypes.data_as(_dp)


def ip(a):
    return a.ctypes.data_as(_ip)


def generate(n, m, seed, lo=-100, hi=100, rand_kind=0, contract=1):
    """(A m x n, b, c) as generateRandomProblem would produce (problem.cu:49-126)."""
    lib = load()
    A_cm = np.zeros(max(n * m, 1))
    b = np.zeros(max(m, 1))
    c = np.zeros(max(n, 1))
    lib.orc_generate_problem(n, m, seed & 0xFFFFFFFF, lo, hi, rand_kind, contract, p(A_cm), p(b), p(c))
    A = A_cm[:n * m].reshape(n, m).T.copy()
    return A, b[:m].copy(), c[:n].copy()


def two_phase(A, b, c, max_pivots=-1):
    lib = load()
    A = np.asarray(A, dtype=np.float64)
    m, n = A.shape
    A_cm = np.ascontiguousarray(A.T).reshape(-1) if n * m else np.zeros(1)
    b = np.ascontiguousarray(b, dtype=np.float64) if m else np.zeros(1)
    c = np.ascontiguousarray(c, dtype=np.float64) if n else np.zeros(1)
    x = np.zeros(max(n, 1))
    opt = ctypes.c_double(0.0)
    p1v = ctypes.c_double(0.0)
    base = np.zeros(max(m, 1), dtype=np.int32)
    piv = np.zeros(2, dtype=np.int64)
    st = lib.orc_two_phase(n, m, p(A_cm), p(b), p(c), max_pivots, p(x), ctypes.byref(opt), ip(base),
                           piv.ctypes.data_as(_lp), ctypes.byref(p1v))
    return {"status": st, "x": x[:n], "opt": opt.value, "base": base[:m], "pivots": (int(piv[0]), int(piv[1])),
            "phase1_value": p1v.value}


def last_objective_row():
    """The last two_phase call's final objective row (as simplex_last_objective_row)."""
    lib = load()
    n = lib.orc_last_objective_row(None, 0)
    d = np.zeros(max(n, 1))
    lib.orc_last_objective_row(p(d), n)
    return d[:n]


def argmin(v):
    lib = load()
    v = np.ascontiguousarray(v, dtype=np.float64)
    vm = ctypes.c_double(0.0)
    i = lib.orc_argmin(p(v), len(v), ctypes.byref(vm))
    return int(i), vm.value


def argmin_tile(v, gidx0):
    lib = load()
    v = np.ascontiguousarray(v, dtype=np.float64)
    pv = ctypes.c_double(0.0)
    pi = ctypes.c_int64(0)
    lib.orc_argmin_tile(p(v), len(v), gidx0, ctypes.byref(pv), ctypes.byref(pi))
    return pv.value, pi.value


def argmin_pass2(pv, pi):
    lib = load()
    pv = np.ascontiguousarray(pv, dtype=np.float64)
    pi = np.ascontiguousarray(pi, dtype=np.int64)
    vm = ctypes.c_double(0.0)
    i = lib.orc_argmin_pass2(p(pv), pi.ctypes.data_as(_lp), len(pv), ctypes.byref(vm))
    return int(i), vm.value


def build_phase1(A, b):
    lib = load()
    m, n = A.shape
    N1 = 1 + n + 2 * m
    A_cm = np.ascontiguousarray(np.asarray(A, dtype=np.float64).T).reshape(-1)
    T = np.zeros((m, N1))
    d = np.zeros(N1)
    base = np.zeros(m, dtype=np.int32)
    lib.orc_build_phase1(n, m, p(A_cm), p(np.ascontiguousarray(b, dtype=np.float64)), p(T), N1, p(d), ip(base))
    return T, d, base


def update_objective(T, d, base):
    lib = load()
    m, ld = T.shape
    lib.orc_update_objective(p(T), m, len(d), ld, ip(base), p(d))


def gemv_partials(T, coef, N):
    lib = load()
    rows, ld = T.shape
    nblk = (rows + 511) // 512
    part = np.zeros((max(nblk, 1), N))
    lib.orc_gemv_partials(p(T), rows, N, ld, p(np.ascontiguousarray(coef)), p(part))
    return part[:nblk]


def gemv_apply(d, partials):
    lib = load()
    partials = np.ascontiguousarray(partials)
    lib.orc_gemv_apply(p(d), len(d), p(partials), partials.shape[0])


def ratio(b, a):
    return load().orc_ratio(b, a)


def apply_update(T, d, prow, colE, r_local, pivot, d_e):
    lib = load()
    rows, ld = T.shape
    N = len(prow)
    lib.orc_apply_update(p(T), rows, N, ld, p(d) if d is not None else None, p(prow), p(colE), r_local, pivot, d_e)


def pivot(T, d, base):
    lib = load()
    m, ld = T.shape
    e = ctypes.c_int64(0)
    r = ctypes.c_int64(0)
    st = lib.orc_pivot(p(T), m, len(d), ld, p(d), ip(base), ctypes.byref(e), ctypes.byref(r))
    return st, e.value, r.value


def solve(T, d, base, max_pivots=-1):
    lib = load()
    m, ld = T.shape
    k = ctypes.c_int64(0)
    st = lib.orc_solve(p(T), m, len(d), ld, p(d), ip(base), max_pivots, ctypes.byref(k))
    return st, k.value


def read_problem_text(path):
    """Python restatement of readProblemFromFile's token order (problem.cu:20-47)."""
    with open(path) as f:
        tok = f.read().split()
    n, m = int(tok[0]), int(tok[1])
    vals = [float(t) for t in tok[2:]]
    c = np.array(vals[:n])
    A = np.zeros((m, n))
    b = np.zeros(m)
    k = n
    for i in range(m):
        A[i] = vals[k:k + n]
        b[i] = vals[k + n]
        k += n + 1
    return A, b, c
