"""HIP path vs CPU oracle, through the C-ABI (needs an MI355X).

Bar: bit-exact on every tableau entry, objective entry, basis and pivot count -- the HIP
kernels perform the same IEEE operations as the reference (fma, correctly rounded
division) in the same order, and the argmin reproduces the reference's combine tree.
"""
import json
import os

import numpy as np
import pytest

import oracle
import simplexoncuda_amd as sx
from conftest import GOLDEN, two_phase_ref

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


def same(a, b):
    return np.array_equal(bits(a), bits(b))


# ------------------------------------------------------------------ argmin tree
@pytest.mark.parametrize("L", [1, 2, 31, 32, 33, 511, 512, 513, 4097, 16384, 73728, 100000])
def test_dev_argmin_matches_oracle(gpu, L):
    rng = np.random.default_rng(L)
    v = rng.integers(-4, 4, size=L).astype(np.float64)
    v[rng.integers(0, L, size=max(1, L // 5))] += rng.choice([3e-10, -7e-10, 2e-9], size=max(1, L // 5))
    assert sx.dev_argmin(v) == oracle.argmin(v)


def test_dev_argmin_all_max(gpu):
    big = np.finfo(np.float64).max
    v = np.full(1000, big)
    assert sx.dev_argmin(v)[0] == -1 == oracle.argmin(v)[0]


# ------------------------------------------------------------------ tableau build + GEMV
@pytest.mark.parametrize("n,m,lo,hi", [(20, 10, 1, 100), (37, 600, -100, 100), (300, 1100, 1, 100), (1, 1, -5, 5)])
def test_build_phase1_bit_exact(gpu, n, m, lo, hi):
    p = sx.generateRandomProblem(n, m, n * 100 + m, lo, hi)
    A, b, c = p.arrays()
    T, d, base = sx.dev_build_phase1(p)
    To, do, bo = oracle.build_phase1(A, b)
    assert same(T, To) and same(d, do) and np.array_equal(base, bo)


@pytest.mark.parametrize("n,m", [(50, 40), (300, 1100)])
def test_update_objective_bit_exact(gpu, n, m):
    A, b, c = oracle.generate(n, m, 7 + n + m, -100, 100)
    T, d, base = oracle.build_phase1(A, b)
    d_gpu = d.copy()
    sx.dev_update_objective(T, d_gpu, base)
    oracle.update_objective(T, d, base)
    assert same(d_gpu, d)


# ------------------------------------------------------------------ pivots
def _phase1_state(n, m, seed, lo=1, hi=100):
    A, b, c = oracle.generate(n, m, seed, lo, hi)
    T, d, base = oracle.build_phase1(A, b)
    oracle.update_objective(T, d, base)
    return T, d, base


@pytest.mark.parametrize("n,m,k", [(20, 10, 5), (256, 256, 40), (333, 1025, 30), (2048, 1024, 25)])
def test_pivots_bit_exact(gpu, n, m, k):
    T, d, base = _phase1_state(n, m, n * 100 + m)
    Tg, dg, bg = T.copy(), d.copy(), base.copy()
    st_g, done_g = sx.dev_pivots(Tg, dg, bg, k)
    st_o, done_o = oracle.solve(T, d, base, max_pivots=k)
    assert done_g == done_o
    assert (st_g == sx.NOT_ENDED) == (st_o == oracle.PIVOT_CAP)
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)


def test_pivots_to_phase_end(gpu):
    T, d, base = _phase1_state(64, 128, 6528)
    Tg, dg, bg = T.copy(), d.copy(), base.copy()
    st_g, done_g = sx.dev_pivots(Tg, dg, bg, 100000)
    st_o, done_o = oracle.solve(T, d, base)
    assert st_g == st_o == oracle.FEASIBLE and done_g == done_o
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)


# ------------------------------------------------------------------ whole two-phase method
def _check_two_phase(p):
    got = sx.twoPhaseMethodEx(p)
    A, b, c = p.arrays()
    ref = two_phase_ref(A, b, c)
    assert got.status == ref["status"]
    assert tuple(got.pivots) == ref["pivots"]
    assert np.array_equal(got.base, ref["base"])
    if got.status == sx.FEASIBLE:
        assert same(got.optimal_value, ref["opt"])
        assert same(got.solution, ref["x"])
    return got, ref


@pytest.mark.parametrize("name", ["smallProblem.txt", "infeasibleProblem.txt", "unboundedProblem.txt"])
def test_examples(gpu, name):
    p = sx.readProblemFromFile(os.path.join(GOLDEN, "examples", name))
    got, _ = _check_two_phase(p)
    expect = {"smallProblem.txt": (sx.FEASIBLE, (2, 2)), "infeasibleProblem.txt": (sx.INFEASIBLE, (2, 0)),
              "unboundedProblem.txt": (sx.UNBOUNDED, (2, 0))}[name]
    assert (got.status, tuple(got.pivots)) == expect
    if got.status == sx.FEASIBLE:
        assert got.optimal_value == pytest.approx(64.0) and list(got.solution) == pytest.approx([8, 0, 0])


@pytest.mark.parametrize("n,m,seed,lo,hi", [
    (20, 10, 2010, 1, 100), (20, 10, 2010, -100, 100), (25, 25, 99, -100, 100), (8, 6, 7, -100, 100),
    (1, 1, 11, 1, 100), (3, 600, 5, 1, 100), (700, 3, 5, 1, 100), (129, 513, 77, -100, 100)])
def test_two_phase_generated(gpu, n, m, seed, lo, hi):
    _check_two_phase(sx.generateRandomProblem(n, m, seed, lo, hi))


def test_two_phase_scipy_optima(gpu):
    with open(os.path.join(GOLDEN, "scipy_optima.json")) as f:
        for r in json.load(f):
            got = sx.twoPhaseMethodEx(sx.generateRandomProblem(r["n"], r["m"], r["seed"], r["lo"], r["hi"]))
            if r["highs_status"] == 0:
                assert got.status == sx.FEASIBLE
                assert got.optimal_value == pytest.approx(r["highs_opt"], rel=1e-6)
            elif r["highs_status"] == 3:
                assert got.status == sx.UNBOUNDED


def _published(n, m):
    with open(os.path.join(GOLDEN, "published_pivots.json")) as f:
        return [x for x in json.load(f) if x["n"] == n and x["m"] == m and x["gpu"] == "rtx2070super"][0]


@pytest.mark.parametrize("n,m", [(256, 256), (1024, 512), (2048, 1024), (8192, 512), (2048, 2048), (8192, 4096)])
def test_published_pivot_counts_on_gpu(gpu, n, m):
    rec = _published(n, m)
    got = sx.twoPhaseMethodEx(sx.generateRandomProblem(n, m, rec["seed"], 1, 100))
    assert got.status == sx.FEASIBLE
    assert tuple(got.pivots) == (rec["p1_pivots"], rec["p2_pivots"])


@pytest.mark.parametrize("fused", [-1, 0])
def test_config2_full_solve_bit_exact(gpu, fused):
    """configs[1]: n=2048, m=1024, seed 205824 -- every bit of the answer vs the oracle."""
    try:
        sx.set_fused(fused)
        got, ref = _check_two_phase(sx.generateRandomProblem(2048, 1024, 205824, 1, 100))
    finally:
        sx.set_fused(-1)
    assert tuple(got.pivots) == (2003, 69)


# ------------------------------------------------------------------ sharded path on one device
@pytest.mark.parametrize("W", [2, 3, 4])
def test_virtual_ranks_pivots_identical(gpu, W):
    T, d, base = _phase1_state(200, 1500, 42)
    ref = (T.copy(), d.copy(), base.copy())
    sx.dev_pivots(*ref, 60)
    try:
        sx.set_virtual_ranks(W)
        Tg, dg, bg = T.copy(), d.copy(), base.copy()
        sx.dev_pivots(Tg, dg, bg, 60)
    finally:
        sx.set_virtual_ranks(1)
    assert same(Tg, ref[0]) and same(dg, ref[1]) and np.array_equal(bg, ref[2])


@pytest.mark.parametrize("W", [2, 8])
def test_virtual_ranks_two_phase(gpu, W):
    """whole two-phase solves on W row-block shards (default exchange): every bit vs the oracle"""
    p = sx.generateRandomProblem(300, 1100, 300 * 100 + 1100, 1, 100)
    try:
        sx.set_virtual_ranks(W)
        _check_two_phase(p)
    finally:
        sx.set_virtual_ranks(1)


# ------------------------------------------------------------------ bench session
def test_session_pivots(gpu):
    p = sx.generateRandomProblem(2048, 1024, 205824, 1, 100)
    sx.set_batch(32)  # (the library reads it at every call)
    try:
        s = sx.Session(p)
        assert s.batch() == 32
        t = s.pivots(50, time_updates=True)
        # 50 pivots = one full batch of 32 + one of 18, each ending with a sweep
        assert t.pivots == 50 and t.status == sx.NOT_ENDED and t.update_launches == 2 and t.swept_pivots == 50
        assert t.update_ms > 0 and t.wall_ms >= t.update_ms
        assert t.stored_width == 1 + 2048 + 1024 and t.width == 1 + 2048 + 2 * 1024
        # slack compaction: a sweep moves 1+n columns plus the slacks of rows that have left
        assert 16.0 * 1024 * (1 + 2048) < t.update_bytes <= 16.0 * 1024 * (1 + 2048 + 50)
        assert t.swept_bytes == 2 * t.update_bytes
        applied, us = s.launch_log()
        assert list(applied) == [32, 18] and (us > 0).all()
        t2 = s.pivots(10000, time_updates=1)
        assert s.total_pivots() == 2003 and t2.status == sx.FEASIBLE
        assert t2.swept_pivots == 2003 - 50  # no-op sweeps after the phase ended are not counted
        s.close()
    finally:
        sx.set_batch(0)


def test_session_two_stage_batches(gpu):
    """64-pivot batches on one shard (the default from 4096 rows): one sweep per batch"""
    p = sx.generateRandomProblem(2048, 1024, 205824, 1, 100)
    sx.set_batch(64)
    try:
        s = sx.Session(p)
        assert s.batch() == 64
        t = s.pivots(150, time_updates=True)
        applied, us = s.launch_log()
        assert t.pivots == 150 and list(applied) == [64, 64, 22] and (us > 0).all()
        t2 = s.pivots(10000)
        assert s.total_pivots() == 2003 and t2.status == sx.FEASIBLE
        s.close()
    finally:
        sx.set_batch(0)
    s2 = sx.Session(generated=(256, 4096, 256 * 100 + 4096, 1, 100))
    assert s2.batch() == 64
    s2.close()


def _pivots_with(cfg, T, d, base, k):
    Tg, dg, bg = T.copy(), d.copy(), base.copy()
    setters = {"batch": (sx.set_batch, 0),
               "fused": (sx.set_fused, -1), "p2p": (sx.set_p2p, -1),
               "waves": (sx.set_update_waves, 0), "W": (sx.set_virtual_ranks, 1),
               "mfma": (sx.set_sweep_mfma, -1), "blocked": (sx.set_blocked, -1)}
    try:
        for key, val in cfg.items():
            setters[key][0](val)
        st, done = sx.dev_pivots(Tg, dg, bg, k)
    finally:
        for key in cfg:
            setters[key][0](setters[key][1])
    return Tg, dg, bg, st, done


@pytest.mark.parametrize("fused", [-1, 0])
@pytest.mark.parametrize("batch", [1, 2, 3, 7, 16, 17, 32])
def test_batched_sweep_bit_exact(gpu, batch, fused):
    """k pivots with the tableau swept every `batch` pivots (pending pivots applied on the fly
    to the columns and rows the decisions read): the same bits as the oracle's pivot-by-pivot
    updates, with a partial last batch; each batch as one resident launch (fused) or as two
    launches per pivot (the default sweep: the matrix cores)"""
    T, d, base = _phase1_state(333, 1025, 7)
    Tg, dg, bg, st, done = _pivots_with({"batch": batch, "fused": fused}, T, d, base, 45)
    oracle.solve(T, d, base, max_pivots=45)
    assert done == 45
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)


@pytest.mark.parametrize("batch", [1, 3, 7, 16, 17])
def test_vector_sweep_slots_bit_exact(gpu, batch):
    """the vector sweep (simplex_set_sweep_mfma(0)) at every register-slot variant (1, 4, 8, 16,
    32 slots) and both row steps (2 rows up to 16 slots, 4 above), with a partial last batch"""
    T, d, base = _phase1_state(333, 1025, 7)
    Tg, dg, bg, st, done = _pivots_with({"batch": batch, "mfma": 0}, T, d, base, 45)
    oracle.solve(T, d, base, max_pivots=45)
    assert done == 45
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)


@pytest.mark.parametrize("batch", [20, 32])
def test_large_batch_sweeps_bit_exact(gpu, batch):
    """the vector sweep's 32-slot variant (batches above 16 pivots), with a partial last batch"""
    T, d, base = _phase1_state(333, 1025, 7)
    Tg, dg, bg, st, done = _pivots_with({"batch": batch, "mfma": 0}, T, d, base, 70)
    oracle.solve(T, d, base, max_pivots=70)
    assert done == 70
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)


@pytest.mark.parametrize("mfma", [1, 0])
@pytest.mark.parametrize("fused", [-1, 0])
@pytest.mark.parametrize("batch", [5, 31])
def test_matrix_core_sweep_bit_exact(gpu, batch, fused, mfma):
    """the sweep on the matrix cores (k_msweep: 4 slots per v_mfma_f64_16x16x4f64, partial
    batches padded, leaving rows recomputed on the vector units) against the vector sweep and the
    oracle: the same bits, 333 rows (a partial 16-row strip), partial last batches"""
    T, d, base = _phase1_state(333, 1025, 7)
    Tg, dg, bg, st, done = _pivots_with({"batch": batch, "fused": fused, "mfma": mfma}, T, d, base, 75)
    oracle.solve(T, d, base, max_pivots=75)
    assert done == 75
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)


@pytest.mark.parametrize("batch", [33, 40, 63, 64])
@pytest.mark.parametrize("inst", [(333, 1025, 7), (300, 1100, 11)])
def test_two_stage_batch_bit_exact(gpu, batch, inst):
    """batches of more than 32 pivots on one shard: the fused batch's second stage (the first
    stage's history in registers, its U / F read back write-through) and the 64-slot matrix-core
    sweep (slots past 32 in PM2), partial last batches: the oracle's bits"""
    T, d, base = _phase1_state(*inst)
    Tg, dg, bg, st, done = _pivots_with({"batch": batch}, T, d, base, 150)
    oracle.solve(T, d, base, max_pivots=150)
    assert done == 150
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)


@pytest.mark.parametrize("n,m,seed,lo,hi", [(64, 128, 6528, 1, 100), (300, 1100, 41100, 1, 100),
                                            (129, 1513, 77, -100, 100), (40, 700, 4070, 1, 100)])
def test_two_stage_batch_whole_phase(gpu, n, m, seed, lo, hi):
    """whole two-phase solves with the default 64-pivot batches (phase ends inside either stage,
    rows leaving in both stages of one batch, slack compaction over two activation passes)"""
    p = sx.generateRandomProblem(n, m, seed, lo, hi)
    sx.set_batch(64)
    try:
        _check_two_phase(p)
    finally:
        sx.set_batch(0)


@pytest.mark.parametrize("W", [2, 4])
def test_matrix_core_sweep_virtual_ranks(gpu, W):
    """the matrix-core sweep on each virtual shard's rows (peer-memory batches, objective tiles
    split across ranks): bit-exact"""
    T, d, base = _phase1_state(300, 1100, 11)
    Tg, dg, bg, st, done = _pivots_with({"batch": 32, "W": W, "p2p": 1, "mfma": 1}, T, d, base, 150)
    st_o, done_o = oracle.solve(T, d, base, max_pivots=150)
    assert done == done_o
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)


@pytest.mark.parametrize("batch", [1, 16, 32, 40, 64])
@pytest.mark.parametrize("W", [2, 3, 4, 8])
def test_p2p_fused_virtual_ranks(gpu, batch, W):
    """the multi-rank fused batch (ranks hand off through each other's memory, objective tiles
    split across ranks): W virtual shards on one GPU, their launches running at once; 40 and 64:
    two-stage batches (the first stage's operands read from U / the owner's F)"""
    T, d, base = _phase1_state(300, 1100, 11)
    Tg, dg, bg, st, done = _pivots_with({"batch": batch, "W": W, "p2p": 1}, T, d, base, 150)
    st_o, done_o = oracle.solve(T, d, base, max_pivots=150)
    assert done == done_o
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)


@pytest.mark.parametrize("batch", [32, 64])
@pytest.mark.parametrize("single", [1, 0])
@pytest.mark.parametrize("W", [2, 3])
def test_p2p_fused_launch_forms(gpu, W, single, batch):
    """the virtual ranks' peer-memory batches as one launch and as one launch per rank on its own
    stream (the RCCL ranks' form): bit-exact, and every batch completed on the fused path (no
    hand-off timed out and fell back to the per-pivot path)"""
    lib = sx.load()
    T, d, base = _phase1_state(300, 1100, 11)
    h0, f0 = lib.simplex_hang_recoveries(), lib.simplex_fused_batches()
    try:
        sx.set_mr_single_launch(single)
        Tg, dg, bg, st, done = _pivots_with({"batch": batch, "W": W, "p2p": 1}, T, d, base, 150)
    finally:
        sx.set_mr_single_launch(1)
    st_o, done_o = oracle.solve(T, d, base, max_pivots=150)
    assert done == done_o
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)
    assert lib.simplex_fused_batches() > f0 and lib.simplex_hang_recoveries() == h0


@pytest.mark.parametrize("W", [2, 3, 8])
@pytest.mark.parametrize("n,m,seed,lo,hi", [(300, 1100, 41100, 1, 100), (129, 1513, 77, -100, 100),
                                            (64, 128, 6528, 1, 100)])
def test_p2p_fused_two_phase(gpu, W, n, m, seed, lo, hi):
    """whole two-phase solves through the multi-rank fused batch, phase ends mid-batch included"""
    p = sx.generateRandomProblem(n, m, seed, lo, hi)
    try:
        sx.set_virtual_ranks(W)
        sx.set_p2p(1)
        _check_two_phase(p)
    finally:
        sx.set_p2p(-1)
        sx.set_virtual_ranks(1)


@pytest.mark.parametrize("W", [2, 3, 8])
@pytest.mark.parametrize("n,m,seed,lo,hi", [(300, 1100, 41100, 1, 100), (129, 1513, 77, -100, 100)])
def test_p2p_fused_two_phase_two_stages(gpu, W, n, m, seed, lo, hi):
    """the same with two-stage (64-pivot) multi-rank batches -- the default from 4096 rows: phase
    ends inside either stage, slack activation in two passes"""
    p = sx.generateRandomProblem(n, m, seed, lo, hi)
    try:
        sx.set_virtual_ranks(W)
        sx.set_p2p(1)
        sx.set_batch(64)
        _check_two_phase(p)
    finally:
        sx.set_batch(0)
        sx.set_p2p(-1)
        sx.set_virtual_ranks(1)


@pytest.mark.parametrize("mfma", [1, 0])
@pytest.mark.parametrize("waves", [1e-4, 0.3, 1, 4])
def test_sweep_grid_bit_exact(gpu, mfma, waves):
    """one block per column tile walking every row group (both directions) up to more blocks
    than row groups; both sweeps"""
    T, d, base = _phase1_state(210, 1700, 3)
    Tg, dg, bg, st, done = _pivots_with({"mfma": mfma, "waves": waves, "batch": 16}, T, d, base, 90)
    oracle.solve(T, d, base, max_pivots=90)
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)


@pytest.mark.parametrize("blocked", [1, 0])
@pytest.mark.parametrize("batch,inst,W", [(5, (333, 1025, 7), 1), (31, (333, 1025, 7), 1), (40, (333, 1025, 7), 1),
                                         (64, (300, 1100, 11), 1), (64, (300, 1100, 11), 4)])
def test_matrix_core_sweep_layouts_bit_exact(gpu, batch, inst, W, blocked):
    """the matrix-core sweep (both tile pairs' four MFMA chains interleaved) on the engine's blocked
    tableau (default) and on row-major storage (simplex_set_blocked(0)): one- and two-stage
    batches, partial ones, virtual shards"""
    T, d, base = _phase1_state(*inst)
    cfg = {"batch": batch, "blocked": blocked, "mfma": 1}
    if W > 1:
        cfg.update({"W": W, "p2p": 1})
    Tg, dg, bg, st, done = _pivots_with(cfg, T, d, base, 150)
    st_o, done_o = oracle.solve(T, d, base, max_pivots=150)
    assert done == done_o
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)


@pytest.mark.parametrize("blocked", [1, 0])
@pytest.mark.parametrize("W", [1, 2, 4])
@pytest.mark.parametrize("n,m,seed,lo,hi", [(300, 1100, 41100, 1, 100), (129, 1513, 77, -100, 100),
                                            (40, 700, 4070, 1, 100), (64, 128, 6528, 1, 100)])
def test_layouts_two_phase(gpu, W, n, m, seed, lo, hi, blocked):
    """whole two-phase solves with the engine's tableaux in 4x4 blocks (the default)
    and row-major (simplex_set_blocked(0)): generator, build, GEMV, both batch kinds, sweeps,
    fix-ups, host transfers and the phase-2 restart address the layout; one shard and virtual
    shards"""
    p = sx.generateRandomProblem(n, m, seed, lo, hi)
    try:
        sx.set_blocked(blocked)
        sx.set_batch(64)
        if W > 1:
            sx.set_virtual_ranks(W)
            sx.set_p2p(1)
        _check_two_phase(p)
    finally:
        sx.set_p2p(-1)
        sx.set_virtual_ranks(1)
        sx.set_batch(0)
        sx.set_blocked(-1)


@pytest.mark.parametrize("blocked", [1, 0])
def test_layouts_two_regions(gpu, blocked):
    """both layouts with the tableau split into two storage regions (the test hook puts 300 slack
    positions in region A)"""
    p = sx.generateRandomProblem(300, 1100, 41100, 1, 100)
    try:
        sx.set_blocked(blocked)
        sx.set_regions(300)
        _check_two_phase(p)
    finally:
        sx.set_regions(1)
        sx.set_blocked(-1)


@pytest.mark.parametrize("fused", [-1, 0])
@pytest.mark.parametrize("batch", [1, 5, 16])
def test_batched_phase_end_mid_batch(gpu, batch, fused):
    """the phase ends inside a batch: the pivots selected before the end are swept, the rest of
    the batch does nothing"""
    T, d, base = _phase1_state(64, 128, 6528)
    Tg, dg, bg, st, done = _pivots_with({"batch": batch, "fused": fused}, T, d, base, 100000)
    st_o, done_o = oracle.solve(T, d, base)
    assert st == st_o == oracle.FEASIBLE and done == done_o
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)


@pytest.mark.parametrize("fused", [-1, 0])
@pytest.mark.parametrize("batch", [1, 16])
def test_same_row_leaves_twice_in_a_batch(gpu, batch, fused):
    """a row that is the leaving row of two pivots of one batch (the general path of the sweep:
    x / p for that slot): on this instance the oracle's leaving rows are 7, 6, 1, 7, 7, 7, ..."""
    T, d, base = _phase1_state(20, 10, 2010)
    ref = (T.copy(), d.copy(), base.copy())
    st_o, done_o = oracle.solve(*ref)
    Tg, dg, bg, st, done = _pivots_with({"batch": batch, "fused": fused}, T, d, base, 100000)
    assert st == st_o and done == done_o
    assert same(Tg, ref[0]) and same(dg, ref[1]) and np.array_equal(bg, ref[2])


@pytest.mark.parametrize("W,case", [(1, (20, 10, 2010, 100000)), (1, (333, 1025, 7, 70)),
                                    (1, (64, 128, 6528, 100000)), (1, (300, 1100, 11, 150)),
                                    (2, (333, 1025, 7, 70)), (2, (300, 1100, 11, 150))])
def test_fused_history_chains(gpu, W, case):
    """the fused batch's pending-pivot chains (ratio rows, pivot row): branch-free when no slot
    of a wave divides, guarded otherwise, one shard and two peer-memory shards; the first
    instance's leaving rows repeat inside a batch (7, 6, 1, 7, 7, 7, ...), so waves of both
    kinds meet in one batch"""
    n, m, seed, k = case
    T, d, base = _phase1_state(n, m, seed)
    ref = (T.copy(), d.copy(), base.copy())
    st_o, done_o = oracle.solve(*ref, max_pivots=k)
    Tg, dg, bg, st, done = _pivots_with({"batch": 32, "W": W, "p2p": 1 if W > 1 else -1}, T, d, base, k)
    assert done == done_o
    assert same(Tg, ref[0]) and same(dg, ref[1]) and np.array_equal(bg, ref[2])


@pytest.mark.parametrize("W,repl", [(1, -1), (2, 0), (2, 1)])
def test_row_leaves_twice_per_stage_compacted(gpu, W, repl):
    """the U invariant the leaving-row restarts rely on (sx_common.hpp Pending::U): a generated
    instance (slack compaction active) whose row 1334 leaves at pivots 394, 420, 427 and 476, 496,
    506 -- twice or more inside both stages of 64-pivot batches (slots 10 / 36 / 43, 28 / 48 / 58) --
    and which lies on shard 1 at W = 2 (rows 1024..1535), while the split objective tiles that form
    its pivot rows sit on both ranks (repl 0) or on every rank (repl 1); 512 pivots against the oracle
    bit for bit, every batch fused"""
    n, m, seed, k = 16, 1536, 142542, 512
    T, d, base = _phase1_state(n, m, seed)
    st_o, done_o = oracle.solve(T, d, base, max_pivots=k)
    lib = sx.load()
    h0, f0 = lib.simplex_hang_recoveries(), lib.simplex_fused_batches()
    bad0 = lib.simplex_pivot_row_mismatches()
    sx.set_virtual_ranks(W)
    sx.set_p2p(1 if W > 1 else -1)
    sx.set_batch(64)
    sx.set_replicated_objective(repl)
    lib.simplex_set_check_pivot_rows(1)
    try:
        sess = sx.Session(generated=(n, m, seed, 1, 100))
        tim = sess.pivots(k)
        act = sess.active_slacks()
        Tg, dg, bg = sess.tableau(m, T.shape[1])
        sess.close()
    finally:
        lib.simplex_set_check_pivot_rows(0)
        sx.set_replicated_objective(-1)
        sx.set_batch(0)
        sx.set_p2p(-1)
        sx.set_virtual_ranks(1)
    assert lib.simplex_pivot_row_mismatches() == bad0  # (every rank's U equal before every sweep)
    assert done_o == k and tim.pivots == k
    assert act < m  # (compaction active: only the slacks of rows that left are swept)
    assert lib.simplex_fused_batches() >= f0 + k // 64 and lib.simplex_hang_recoveries() == h0
    assert np.array_equal(bg, base) and same(dg, d) and same(Tg, T)


@pytest.mark.parametrize("batch", [4, 16])
@pytest.mark.parametrize("W", [2, 3])
def test_batched_virtual_ranks(gpu, batch, W):
    T, d, base = _phase1_state(300, 1100, 11)
    Tg, dg, bg, st, done = _pivots_with({"batch": batch, "W": W}, T, d, base, 120)
    oracle.solve(T, d, base, max_pivots=120)
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)


@pytest.mark.parametrize("W", [1, 2, 3])
@pytest.mark.parametrize("mode", [1, 2])
def test_exchange_path_bit_exact(gpu, W, mode):
    """the multi-shard kernels on virtual shards (W=1 runs them with a single shard):
    mode 1 = tile allgather + select/row copy + -0.0 allreduce; mode 2 = one allgather of
    tile winners with their rows + single-block select"""
    p = sx.generateRandomProblem(300, 1100, 300 * 100 + 1100, 1, 100)
    try:
        sx.set_virtual_ranks(W)
        sx.set_force_exchange(1)
        sx.set_exchange_mode(mode)
        got, _ = _check_two_phase(p)
    finally:
        sx.set_exchange_mode(0)
        sx.set_force_exchange(0)
        sx.set_virtual_ranks(1)
    assert got.status == sx.FEASIBLE


def test_rccl_one_rank_multirank_paths(gpu):
    """the multi-GPU code paths over a REAL RCCL communicator (1 rank): the peer-memory fused
    batch with its IPC-handle exchange, and both per-pivot RCCL exchanges -- whole solves
    bit-exact vs the oracle (child process: the library's distributed state is process-global)"""
    import subprocess
    import sys
    from conftest import ROOT
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "rccl_one_rank.py")], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "ALL BIT-EXACT" in r.stdout and r.stdout.count("bit-exact") == 9


def test_c_caller_drop_in(gpu, tmp_path):
    """a reference-style C program linked against libsimplex_hip.so solves smallProblem.txt"""
    import subprocess
    from test_abi import _build_c_caller
    exe = _build_c_caller(tmp_path, "gcc", "c99")
    r = subprocess.run([str(exe), "solve", os.path.join(GOLDEN, "examples", "smallProblem.txt")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "status 0 z 64.000000 x0 8.000000" in r.stdout


@pytest.mark.parametrize("alias", [0, 1])
def test_alias_storage_on_off(gpu, alias):
    """phase-1 artificial columns stored as their slack columns (default) or explicitly:
    identical bits either way"""
    p = sx.generateRandomProblem(129, 513, 77, -100, 100)
    try:
        sx.set_alias(alias)
        _check_two_phase(p)
        T, d, base = _phase1_state(200, 700, 5)
        Tg, dg, bg = T.copy(), d.copy(), base.copy()
        sx.dev_pivots(Tg, dg, bg, 40)
        oracle.solve(T, d, base, max_pivots=40)
        assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)
    finally:
        sx.set_alias(1)


def test_pivots_without_alias_invariant(gpu):
    """a tableau whose artificial columns differ from the slack columns is stored in full"""
    T, d, base = _phase1_state(100, 300, 9)
    n, m = 100, 300
    T[5, 1 + n + m + 7] += 0.25  # break the artificial == slack invariant
    Tg, dg, bg = T.copy(), d.copy(), base.copy()
    sx.dev_pivots(Tg, dg, bg, 30)
    oracle.solve(T, d, base, max_pivots=30)
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)


@pytest.mark.parametrize("lo", [-100, 1])
def test_negative_zeros_kept(gpu, lo):
    """a tableau holding -0.0 (the b<0 row negation of the build, or a caller's upload):
    fma(0, p, -0.0) is +0.0, and every element is swept exactly as the reference does"""
    T, d, base = _phase1_state(200, 700, 5, lo, 100)
    if lo > 0:
        T[T == 0.0] = -0.0
    assert np.signbit(T[T == 0.0]).any()
    Tg, dg, bg = T.copy(), d.copy(), base.copy()
    sx.dev_pivots(Tg, dg, bg, 60)
    oracle.solve(T, d, base, max_pivots=60)
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)


def test_two_phase_negated_rows(gpu):
    """generated instances with b_i < 0 (values in [-100, 100]): host and device builds"""
    p = sx.generateRandomProblem(150, 700, 1234, -100, 100)
    _check_two_phase(p)
    s = sx.Session(generated=(150, 700, 1234, -100, 100))
    t = s.pivots(40, time_updates=1)
    assert t.pivots == 40 and t.swept_pivots == 40
    s.close()


# ------------------------------------------------------------------ slack compaction
def _oracle_after(p, k):
    A, b, c = p.arrays()
    T, d, base = oracle.build_phase1(A, b)
    oracle.update_objective(T, d, base)
    _, done = oracle.solve(T, d, base, max_pivots=k)
    return T, d, base, done


@pytest.mark.parametrize("compact", [1, 0])
@pytest.mark.parametrize("n,m,k,fused,W,p2p", [
    (300, 1100, 200, -1, 1, -1),   # fused batches
    (300, 1100, 200, 0, 1, -1),    # per-pivot launches
    (64, 700, 400, -1, 1, -1),     # many pivots per row: rows leave again
    (200, 1500, 150, -1, 2, 0),    # two shards, RCCL-style exchange
    (200, 1500, 150, -1, 2, 1),    # two shards, fused batches over peer memory
])
def test_slack_compaction_tableau_bit_exact(gpu, n, m, k, fused, W, p2p, compact):
    """sweeps that skip the untouched slack columns leave every logical entry of the
    tableau -- the untouched unit vectors included -- bit-identical to the oracle's"""
    p = sx.generateRandomProblem(n, m, n * 100 + m, 1, 100)
    try:
        sx.set_compact(compact)
        sx.set_fused(fused)
        sx.set_p2p(p2p)
        sx.set_virtual_ranks(W)
        s = sx.Session(problem=p)
        t = s.pivots(k)
        Tg, dg, bg = s.tableau(m, 1 + n + 2 * m)
        active = s.active_slacks()
        s.close()
    finally:
        sx.set_virtual_ranks(1)
        sx.set_p2p(-1)
        sx.set_fused(-1)
        sx.set_compact(1)
    T, d, base, done = _oracle_after(p, k)
    assert t.pivots == done
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)
    if compact:
        assert 0 < active <= done and active < m
    else:
        assert active == m


@pytest.mark.parametrize("cap", [16, 300])
@pytest.mark.parametrize("n,m,k,fused,W,p2p", [
    (300, 1100, 200, -1, 1, -1),   # fused batches
    (300, 1100, 200, 0, 1, -1),    # per-pivot launches
    (64, 700, 400, -1, 1, -1),     # rows leave again; the swept block grows past region A
    (200, 1500, 150, -1, 2, 0),    # two shards, RCCL-style exchange
    (200, 1500, 150, -1, 2, 1),    # two shards, fused batches over peer memory
])
def test_two_region_layout_bit_exact(gpu, n, m, k, fused, W, p2p, cap):
    """the two-region tableau layout (region A: structural columns + the first `cap` stored
    slack positions, region B: the rest) with a small region A, so activations, leaving-row and
    entering-column reads and sweeps all cross into region B: every logical entry bit-identical
    to the oracle's"""
    p = sx.generateRandomProblem(n, m, n * 100 + m, 1, 100)
    try:
        sx.set_regions(cap)
        sx.set_fused(fused)
        sx.set_p2p(p2p)
        sx.set_virtual_ranks(W)
        s = sx.Session(problem=p)
        t = s.pivots(k)
        Tg, dg, bg = s.tableau(m, 1 + n + 2 * m)
        active = s.active_slacks()
        s.close()
    finally:
        sx.set_virtual_ranks(1)
        sx.set_p2p(-1)
        sx.set_fused(-1)
        sx.set_regions(1)
    T, d, base, done = _oracle_after(p, k)
    assert t.pivots == done
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)
    assert 0 < active <= done


@pytest.mark.parametrize("W,p2p", [(1, -1), (2, 1), (3, 0)])
@pytest.mark.parametrize("n,m,seed,lo,hi", [(300, 1100, 41100, 1, 100), (64, 128, 6528, 1, 100),
                                            (129, 1513, 77, -100, 100)])
@pytest.mark.parametrize("mfma", [0, 1])
def test_two_region_two_phase(gpu, n, m, seed, lo, hi, W, p2p, mfma):
    """whole two-phase solves (GEMV, phase switch, solution) on the two-region layout with a
    region A of 16 slack positions, on 1-3 shards, swept on the vector units or the matrix cores"""
    p = sx.generateRandomProblem(n, m, seed, lo, hi)
    try:
        sx.set_regions(16)
        sx.set_virtual_ranks(W)
        sx.set_p2p(p2p)
        sx.set_sweep_mfma(mfma)
        _check_two_phase(p)
    finally:
        sx.set_sweep_mfma(-1)
        sx.set_p2p(-1)
        sx.set_virtual_ranks(1)
        sx.set_regions(1)


def test_slack_compaction_off_for_negated_rows(gpu):
    """a b < 0 row is negated at build (its -0.0 entries could flip a zero's sign in an
    untouched column): no compaction, still bit-exact"""
    p = sx.generateRandomProblem(150, 700, 1234, -100, 100)
    s = sx.Session(problem=p)
    s.pivots(60)
    Tg, dg, bg = s.tableau(700, 1 + 150 + 1400)
    assert s.active_slacks() == 700
    s.close()
    T, d, base, _ = _oracle_after(p, 60)
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)


def test_slack_compaction_generated_session_width(gpu):
    """device-built tableau: the timed sweeps move 1+n+(swept slacks) columns -- at most the slacks
    of the rows that have left (<= the pivots), fewer once basic slacks leave the sweep"""
    n, m = 512, 2048
    s = sx.Session(generated=(n, m, n * 100 + m, 1, 100))
    K = s.batch()
    assert K == 32  # (the default below 4096 rows)
    t = s.pivots(96, time_updates=1)
    active = s.active_slacks()
    s.close()
    assert 0 < active <= 96
    assert t.update_launches == (96 + K - 1) // K and t.swept_pivots == 96
    assert t.update_bytes <= 16.0 * m * (1 + n + 96) + 1e-6
    assert t.update_bytes < 16.0 * m * t.stored_width


# ------------------------------------------------------------------ round 4
@pytest.mark.parametrize("batch", [32, 64])
@pytest.mark.parametrize("W", [2, 8])
def test_p2p_fused_fine_pivot_rows(gpu, batch, W):
    """the pending pivot rows U in fine-grained memory -- what the engine allocates when the shards
    span devices (peer ranks write U over xGMI) -- forced on one GPU: the multi-rank
    batch and its sweeps stay bit-exact"""
    lib = sx.load()
    T, d, base = _phase1_state(300, 1100, 11)
    try:
        lib.simplex_set_fine_pivot_rows(1)
        Tg, dg, bg, st, done = _pivots_with({"batch": batch, "W": W, "p2p": 1}, T, d, base, 150)
    finally:
        lib.simplex_set_fine_pivot_rows(-1)
    st_o, done_o = oracle.solve(T, d, base, max_pivots=150)
    assert done == done_o
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)


def _subnormal_state(seed):
    """a phase-1 state whose structural block holds IEEE edge values the pivot decisions do not
    depend on: subnormals, entries of 1e-300 scale (their products with the row factors underflow
    to subnormals or zero) and signed zeros, ~12 % of the structural entries"""
    n, m = 300, 1100
    T, d, base = _phase1_state(n, m, seed)
    rng = np.random.default_rng(seed)
    blk = T[:, 1:1 + n]
    pick = rng.random(blk.shape)
    sub = rng.integers(1, 1 << 52, size=blk.shape, dtype=np.uint64).view(np.float64)
    tiny = rng.uniform(-1.0, 1.0, size=blk.shape) * 1e-300
    blk[pick < 0.04] = sub[pick < 0.04] * np.where(rng.random(blk.shape) < 0.5, -1.0, 1.0)[pick < 0.04]
    blk[(pick >= 0.04) & (pick < 0.08)] = tiny[(pick >= 0.04) & (pick < 0.08)]
    blk[(pick >= 0.08) & (pick < 0.10)] = -0.0
    blk[(pick >= 0.10) & (pick < 0.12)] = 0.0
    # ~5 % of the rows scaled into the subnormal range (RHS included): their entering entries stay
    # below the 1e-9 eligibility bound, so they never leave, and their factors and updates stay
    # subnormal pivot after pivot
    rows = rng.random(m) < 0.05
    T[rows, :1 + n] *= 2.0 ** -1040
    return T, d, base


@pytest.mark.parametrize("batch,mfma", [(64, 1), (32, 1), (17, 1), (32, 0)])
def test_subnormal_tableau_bit_exact(gpu, batch, mfma):
    """the sweep on a tableau holding subnormal, underflowing and signed-zero entries: the matrix
    cores (v_mfma_f64_16x16x4f64: 64- and 32-slot sweeps, a partial batch) and the vector units
    give the oracle's per-element fma chain bit for bit -- the edge semantics the matrix-core sweep
    depends on (profiles/r04_mfma_edge_probe.txt), here through the engine"""
    T, d, base = _subnormal_state(11)
    sub0 = np.count_nonzero((T != 0) & (np.abs(T) < 2.2250738585072014e-308))
    assert sub0 > 1000
    Tg, dg, bg, st, done = _pivots_with({"batch": batch, "mfma": mfma}, T, d, base, 130)
    st_o, done_o = oracle.solve(T, d, base, max_pivots=130)
    assert done == done_o
    assert np.count_nonzero((T != 0) & (np.abs(T) < 2.2250738585072014e-308)) > 1000  # (subnormal results too)
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)


# ------------------------------------------------------------------ round 5
@pytest.mark.parametrize("batch", [32, 64])
@pytest.mark.parametrize("W", [2, 3, 4, 8])
def test_replicated_objective_pivots(gpu, batch, W):
    """multi-rank fused batches with the objective row replicated (every rank runs every objective
    tile, decides the entering variable from its own records and forms the whole pivot row in its
    own U; simplex_set_replicated_objective) on W virtual shards: bit-exact with the
    oracle, every batch fused, no hang recovery"""
    lib = sx.load()
    T, d, base = _phase1_state(300, 1100, 11)
    f0, h0 = lib.simplex_fused_batches(), lib.simplex_hang_recoveries()
    try:
        sx.set_replicated_objective(1)
        Tg, dg, bg, st, done = _pivots_with({"batch": batch, "W": W, "p2p": 1}, T, d, base, 150)
    finally:
        sx.set_replicated_objective(-1)
    st_o, done_o = oracle.solve(T, d, base, max_pivots=150)
    assert done == done_o
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)
    assert lib.simplex_fused_batches() - f0 >= 150 // batch
    assert lib.simplex_hang_recoveries() == h0


@pytest.mark.parametrize("W", [2, 4])
@pytest.mark.parametrize("n,m,seed,lo,hi", [(300, 1100, 5, 1, 100), (200, 1500, 77, -100, 100)])
def test_replicated_objective_two_phase(gpu, W, n, m, seed, lo, hi):
    """whole two-phase solves (phase 2's narrower row included; the second instance negates rows:
    no slack compaction) on virtual shards with the replicated objective"""
    p = sx.generateRandomProblem(n, m, seed, lo, hi)
    try:
        sx.set_replicated_objective(1)
        sx.set_virtual_ranks(W)
        sx.set_p2p(1)
        _check_two_phase(p)
    finally:
        sx.set_p2p(-1)
        sx.set_virtual_ranks(1)
        sx.set_replicated_objective(-1)


@pytest.mark.parametrize("slot", [3, 40])
def test_replicated_objective_hang_recovery(gpu, slot):
    """a replicated multi-rank batch aborted from inside after `slot` pivots (the objective row
    already updated by them on every rank): each rank restores its whole row and the batch is
    re-run on the per-pivot path -- still bit-exact"""
    lib = sx.load()
    T, d, base = _phase1_state(300, 1100, 11)
    h0 = lib.simplex_hang_recoveries()
    try:
        sx.set_replicated_objective(1)
        lib.simplex_set_hang_inject(1)
        lib.simplex_set_hang_inject_slot(slot)
        Tg, dg, bg, st, done = _pivots_with({"batch": 64, "W": 2, "p2p": 1}, T, d, base, 150)
    finally:
        lib.simplex_set_hang_inject(-1)
        lib.simplex_set_hang_inject_slot(-1)
        sx.set_replicated_objective(-1)
    st_o, done_o = oracle.solve(T, d, base, max_pivots=150)
    assert done == done_o
    assert same(Tg, T) and same(dg, d) and np.array_equal(bg, base)
    assert lib.simplex_hang_recoveries() == h0 + 1
