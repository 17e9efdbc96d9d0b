"""The inner drop-in entry point on a caller-built tableau, through a C program:
newTabular (tabular.cu:25-39) -> fill table / costsVector -> solve (solver.cu:128-149) ->
read back -> freeTabular, compared bit for bit with the CPU oracle's solve on the same state.
"""
import os
import subprocess

import numpy as np
import pytest

import oracle
from conftest import ROOT

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


@pytest.fixture(scope="module")
def caller(tmp_path_factory):
    exe = tmp_path_factory.mktemp("tabular") / "tabular_main"
    lib = os.path.join(ROOT, "simplexoncuda_amd")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "c", "tabular_main.c"),
                    "-L", lib, "-lsimplex_hip", "-L/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{lib}",
                    "-Wl,-rpath,/opt/rocm/lib", "-o", str(exe)], check=True)
    return exe


def run_caller(exe, tmp_path, n, m, T, d, base):
    """-> (status, rows, cols, pitch, T, d, base) after the C program's solve()."""
    m_, W = T.shape
    assert m_ == m and len(d) == W
    fin, fout = tmp_path / "in.bin", tmp_path / "out.bin"
    with open(fin, "wb") as f:
        f.write(np.array([n, m, W], dtype=np.int32).tobytes())
        f.write(np.ascontiguousarray(T, dtype=np.float64).tobytes())
        f.write(np.ascontiguousarray(d, dtype=np.float64).tobytes())
        f.write(np.ascontiguousarray(base, dtype=np.int32).tobytes())
    r = subprocess.run([str(exe), str(fin), str(fout)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = fout.read_bytes()
    st, rows, cols = np.frombuffer(raw[:12], dtype=np.int32)
    pitch = int(np.frombuffer(raw[12:20], dtype=np.int64)[0])
    off = 20
    To = np.frombuffer(raw[off:off + 8 * m * W], dtype=np.float64).reshape(m, W)
    off += 8 * m * W
    do = np.frombuffer(raw[off:off + 8 * W], dtype=np.float64)
    off += 8 * W
    bo = np.frombuffer(raw[off:off + 4 * m], dtype=np.int32)
    return int(st), int(rows), int(cols), pitch, To, do, bo


def phase1(n, m, seed, lo, hi):
    A, b, c = oracle.generate(n, m, seed, lo, hi)
    T, d, base = oracle.build_phase1(A, b)
    oracle.update_objective(T, d, base)
    return A, b, c, T, d, base


def check(exe, tmp_path, n, m, T, d, base):
    got = run_caller(exe, tmp_path, n, m, T.copy(), d.copy(), base.copy())
    st_o, _ = oracle.solve(T, d, base)
    st, rows, cols, pitch, Tg, dg, bg = got
    assert st == st_o
    assert rows == T.shape[1] and cols == m and pitch >= 8 * (1 + n + 2 * m)
    assert np.array_equal(bits(Tg), bits(T))
    assert np.array_equal(bits(dg), bits(d))
    assert np.array_equal(bg, base)
    return st


@pytest.mark.parametrize("n,m,seed,lo,hi", [(20, 10, 2010, 1, 100), (60, 90, 7, -100, 100),
                                            (300, 700, 11, 1, 100), (129, 1513, 77, -100, 100)])
def test_tabular_phase1_solve(gpu, caller, tmp_path, n, m, seed, lo, hi):
    _, _, _, T, d, base = phase1(n, m, seed, lo, hi)
    check(caller, tmp_path, n, m, T, d, base)


@pytest.mark.parametrize("n,m,seed", [(20, 10, 2010), (300, 700, 11)])
def test_tabular_phase2_solve(gpu, caller, tmp_path, n, m, seed):
    """phase 2 as twoPhaseMethod.cu:285-356 drives it: rows -= cols, costs -c / 0 (d[0] kept),
    objective canonicalised, then solve"""
    A, b, c, T, d, base = phase1(n, m, seed, 1, 100)
    st1, _ = oracle.solve(T, d, base)
    assert st1 == oracle.FEASIBLE
    N2 = 1 + n + m
    T2 = np.ascontiguousarray(T[:, :N2])
    d2 = d[:N2].copy()
    d2[1:1 + n] = -c
    d2[1 + n:] = 0.0
    oracle.update_objective(T2, d2, base)
    check(caller, tmp_path, n, m, T2, d2, base)


def test_tabular_artificials_not_slacks(gpu, caller, tmp_path):
    """a caller's tableau whose artificial columns are not copies of the slack columns (the
    engine's aliased storage could not hold it): stored in full, solved exactly"""
    n, m = 40, 64
    _, _, _, T, d, base = phase1(n, m, 99, 1, 100)
    rng = np.random.default_rng(5)
    T[:, 1 + n + m:] += rng.uniform(0.0, 0.5, size=(m, m))
    check(caller, tmp_path, n, m, T, d, base)
