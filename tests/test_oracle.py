"""The CPU oracle against the reference's own pins (CPU only)."""
import json
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN

EX = os.path.join(GOLDEN, "examples")


def _published():
    with open(os.path.join(GOLDEN, "published_pivots.json")) as f:
        return json.load(f)


# Appendix C of SURVEY.md: hand-traced answers for data/examples/*.txt
def test_small_problem_known_answer():
    A, b, c = oracle.read_problem_text(os.path.join(EX, "smallProblem.txt"))
    r = oracle.two_phase(A, b, c)
    assert r["status"] == oracle.FEASIBLE
    assert r["opt"] == pytest.approx(64.0, rel=1e-12)
    assert np.allclose(r["x"], [8.0, 0.0, 0.0])
    assert list(r["base"]) == [3, 0]
    assert r["pivots"] == (2, 2)


def test_unbounded_problem_known_answer():
    A, b, c = oracle.read_problem_text(os.path.join(EX, "unboundedProblem.txt"))
    r = oracle.two_phase(A, b, c)
    assert r["status"] == oracle.UNBOUNDED
    assert r["pivots"] == (2, 0)


def test_infeasible_problem_known_answer():
    A, b, c = oracle.read_problem_text(os.path.join(EX, "infeasibleProblem.txt"))
    r = oracle.two_phase(A, b, c)
    assert r["status"] == oracle.INFEASIBLE
    assert r["pivots"][0] == 2
    assert r["phase1_value"] == pytest.approx(-5.0, abs=1e-12)


# data/measures line counts (tests/golden/published_pivots.json): the instances the CPU
# oracle finishes in seconds.  They pin generator, tie-breaking and arithmetic together.
FAST = [(256, 256), (512, 256), (256, 512), (1024, 256), (512, 512), (2048, 256), (4096, 256)]


@pytest.mark.parametrize("n,m", FAST)
def test_published_pivot_counts(n, m):
    rec = [x for x in _published() if x["n"] == n and x["m"] == m and x["gpu"] == "rtx2070super"][0]
    A, b, c = oracle.generate(n, m, rec["seed"], 1, 100)
    r = oracle.two_phase(A, b, c)
    assert r["status"] == oracle.FEASIBLE
    assert r["pivots"] == (rec["p1_pivots"], rec["p2_pivots"])


def test_published_counts_identical_across_gpus_but_one():
    recs = _published()
    by = {}
    for x in recs:
        by.setdefault((x["n"], x["m"]), {})[x["gpu"]] = x
    diff = [k for k, v in by.items()
            if (v["rtx2070super"]["p1_pivots"], v["rtx2070super"]["p2_pivots"])
            != (v["mx250_2"]["p1_pivots"], v["mx250_2"]["p2_pivots"])]
    assert len(by) == 36 and diff == [(1024, 8192)]


@pytest.mark.slow
@pytest.mark.parametrize("n,m", [(2048, 1024)])
def test_published_pivot_counts_config2(n, m):
    rec = [x for x in _published() if x["n"] == n and x["m"] == m and x["gpu"] == "rtx2070super"][0]
    A, b, c = oracle.generate(n, m, rec["seed"], 1, 100)
    r = oracle.two_phase(A, b, c)
    assert r["pivots"] == (rec["p1_pivots"], rec["p2_pivots"]) == (2003, 69)


def test_scipy_highs_optima():
    with open(os.path.join(GOLDEN, "scipy_optima.json")) as f:
        cases = json.load(f)
    for r in cases:
        A, b, c = oracle.generate(r["n"], r["m"], r["seed"], r["lo"], r["hi"])
        o = oracle.two_phase(A, b, c)
        if r["highs_status"] == 0:
            assert o["status"] == oracle.FEASIBLE
            assert o["opt"] == pytest.approx(r["highs_opt"], rel=1e-6)
        elif r["highs_status"] == 3:
            assert o["status"] == oracle.UNBOUNDED


# ---- the epsilon argmin tree (reduction.cu:10-104) ----
def _py_argmin(v):
    """Pure-Python restatement of the two-pass tree for small vectors."""
    big = np.finfo(np.float64).max

    def cmp(x, y):
        if abs(x - y) < 1e-9:
            return 0
        return -1 if x < y else 1

    def warp(l):
        l = list(l)
        off = 16
        while off:
            for k in range(32 - off):
                if cmp(l[k + off][0], l[k][0]) < 0:
                    l[k] = l[k + off]
            off //= 2
        return l[0]

    def block(th):
        nw = len(th) // 32
        win = [warp(th[w * 32:(w + 1) * 32]) for w in range(nw)]
        win += [(big, -1)] * (32 - nw)
        return warp(win)

    L = len(v)
    grid = max(1, min((L + 511) // 512, 1024))
    parts = []
    for bi in range(grid):
        th = []
        for t in range(512):
            cur = (big, -1)
            i = bi * 512 + t
            while i < L:
                if cmp(v[i], cur[0]) < 0:
                    cur = (v[i], i)
                i += 512 * grid
            th.append(cur)
        parts.append(block(th))
    if grid == 1:
        return parts[0][1], parts[0][0]
    th = []
    for t in range(1024):
        cur = (big, -1)
        if t < grid and cmp(parts[t][0], cur[0]) < 0:
            cur = parts[t]
        th.append(cur)
    w = block(th)
    return w[1], w[0]


@pytest.mark.parametrize("L", [1, 31, 32, 33, 511, 512, 513, 1500, 4097])
def test_argmin_tree_matches_python_restatement(L):
    rng = np.random.default_rng(L)
    v = rng.integers(-3, 3, size=L).astype(np.float64)  # many exact ties
    v[rng.integers(0, L, size=max(1, L // 7))] += 5e-10  # epsilon ties
    assert oracle.argmin(v) == _py_argmin(v)


def test_argmin_tie_is_not_lowest_index():
    v = np.zeros(64)
    v[[1, 2]] = -1.0  # lanes 1 and 2 tie exactly: lane 2 wins (bit-reversed lane order)
    assert oracle.argmin(v)[0] == 2
    v = np.zeros(600)
    v[[3, 520]] = -1.0  # tie across tiles: tile 0 keeps its winner
    assert oracle.argmin(v)[0] == 3


def test_argmin_epsilon_nonassociative():
    # x1 within eps of x0 and x2 within eps of x1 but x2 < x0 - eps: order decides
    v = np.array([0.0, -0.6e-9, -1.2e-9] + [1.0] * 29)
    i, _ = oracle.argmin(v)
    assert i == _py_argmin(v)[0]


def test_ratio_vector_entries():
    big = np.finfo(np.float64).max
    assert oracle.ratio(4.0, 2.0) == 2.0
    assert oracle.ratio(4.0, 5e-10) == big      # |a| < eps: not eligible
    assert oracle.ratio(4.0, -1.0) == big
    assert oracle.ratio(-4.0, 2.0) == -2.0      # negative RHS from rounding is kept


def test_phase1_build_b_negative_quirk():
    A = np.array([[1.0, 2.0], [3.0, 4.0]])
    b = np.array([5.0, -6.0])
    T, d, base = oracle.build_phase1(A, b)
    # row 1 negated across everything, slack and artificial included (twoPhaseMethod.cu:86-111)
    assert list(T[1]) == [6.0, -3.0, -4.0, -0.0, -1.0, -0.0, -1.0]
    assert np.signbit(T[1][3]) and np.signbit(T[1][5])
    assert list(base) == [4, 5]
    assert list(d) == [0, 0, 0, 0, 0, 1, 1]


# DEGENERATE (-3) pins: tests/golden/degenerate_cases.json (scripts/make_degenerate_cases.py)
def test_degenerate_fixtures_reproduced():
    with open(os.path.join(GOLDEN, "degenerate_cases.json")) as f:
        cases = json.load(f)
    for s in cases["small"]:
        r = oracle.two_phase(np.array(s["A"]), np.array(s["b"]), np.array(s["c"]))
        assert r["status"] == oracle.DEGENERATE == s["status"]
        assert list(r["pivots"]) == s["pivots"] and r["base"].tolist() == s["base"]
    e = cases["embedded"][0]
    nb, mb, seed = e["big"]
    s = cases["small"][e["small"]]
    Ab, bb, cb = oracle.generate(nb, mb, seed, 1, 100)
    As = np.array(s["A"])
    A = np.zeros((mb + As.shape[0], nb + As.shape[1]))
    A[:mb, :nb] = Ab
    A[mb:, nb:] = As
    r = oracle.two_phase(A, np.concatenate([bb, s["b"]]), np.concatenate([cb, s["c"]]))
    assert r["status"] == oracle.DEGENERATE and list(r["pivots"]) == e["pivots"]


# SURVEY.md §5 race/sanitizer row: the oracle built with -fsanitize=address,undefined
# (oracle/Makefile `sanitize`) runs the examples and generated instances cleanly and agrees
# with the plain build
def test_oracle_under_sanitizers(tmp_path):
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(os.path.dirname(GOLDEN), "..", "oracle"), "sanitize"],
                   check=True)
    exe = os.path.join(os.path.dirname(GOLDEN), "..", "oracle", "oracle_cli_san")
    with open(os.path.join(GOLDEN, "degenerate_cases.json")) as f:
        s = json.load(f)["small"][0]
    deg = tmp_path / "degenerate.txt"  # readProblemFromFile format (problem.cu:20-47)
    A, b, c = np.array(s["A"]), np.array(s["b"]), np.array(s["c"])
    lines = [f"{A.shape[1]} {A.shape[0]}", " ".join(repr(float(v)) for v in c)]
    lines += [" ".join(repr(float(v)) for v in list(A[i]) + [b[i]]) for i in range(A.shape[0])]
    deg.write_text("\n".join(lines) + "\n")
    runs = [["file", os.path.join(EX, f)] for f in ("smallProblem.txt", "infeasibleProblem.txt",
                                                    "unboundedProblem.txt")]
    runs += [["file", str(deg)], ["gen", "20", "10", "2010"], ["gen", "256", "256", "25856"],
             ["gen", "37", "600", "5", "-100", "100"]]
    expect = {"smallProblem.txt": "0 2 2", "infeasibleProblem.txt": "-1 2 0", "unboundedProblem.txt": "-2 2 0",
              "degenerate.txt": f"-3 {s['pivots'][0]} {s['pivots'][1]}", "25856": "0 459 25"}
    for args in runs:
        r = subprocess.run([exe] + args, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0 and "Sanitizer" not in r.stderr, r.stderr[-2000:]
        key = os.path.basename(args[1]) if args[0] == "file" else args[3]
        if key in expect:
            assert r.stdout.startswith(expect[key]), (key, r.stdout)
