"""Basic slack columns moved out of the sweep (k_deact_* in sx_kernels.hip).

A slack that enters the basis leaves its column the unit vector e_r where the residuals
a_k - fl(a_k / p) p of the reference's pivot (solver.cu:34-46) round to +0 (checked bit for bit), and
later pivots leave it bit-identical until its row leaves again; with slack compaction such columns
are moved behind the swept block every few
sweeps and moved back when their row leaves.  Every logical entry of the tableau must stay the
oracle's, through re-entries and re-activations, on the fused and the per-pivot paths (one shard),
and the whole two-phase method must return the oracle's answer (needs an MI355X).
"""
import numpy as np
import pytest

import oracle
import simplexoncuda_amd as sx
from conftest import two_phase_ref

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


def same(a, b):
    return np.array_equal(bits(a), bits(b))


def _oracle_after(p, k):
    A, b, c = p.arrays()
    T, d, base = oracle.build_phase1(A, b)
    oracle.update_objective(T, d, base)
    _, done = oracle.solve(T, d, base, max_pivots=k)
    return T, d, base, done


def _session_run(p, stops, deact, fused, batch):
    """the tableau, objective row, basis and swept slack count at each stop"""
    out = []
    try:
        sx.set_deactivate(deact)
        sx.set_fused(fused)
        sx.set_batch(batch)
        s = sx.Session(problem=p)
        for k in stops:
            t = s.pivots(k - s.total_pivots())
            Tg, dg, bg = s.tableau(p.m, 1 + p.n + 2 * p.m)
            out.append((t.status, s.total_pivots(), Tg, dg, bg, s.active_slacks()))
            if t.status != sx.NOT_ENDED:
                break
        s.close()
    finally:
        sx.set_batch(0)
        sx.set_fused(-1)
        sx.set_deactivate(sx.DEACTIVATE_EVERY)
    return out


@pytest.mark.parametrize("every", [1, 3])
@pytest.mark.parametrize("n,m,stops,fused,batch", [
    (64, 700, (150, 400, 700), -1, 0),     # fused batches (32 pivots below 4096 rows)
    (64, 700, (150, 400, 700), 0, 0),      # per-pivot launches + k_activate
    (64, 700, (200, 700), -1, 64),         # two-stage batches
    (300, 1100, (300, 900), -1, 64),
    (16, 1536, (500, 1200), -1, 64),       # few structurals: the slacks re-enter quickly
])
def test_deactivated_slacks_tableau_bit_exact(gpu, n, m, stops, fused, batch, every):
    """(every: sweeps between two rounds of moving basic slacks out)"""
    p = sx.generateRandomProblem(n, m, n * 100 + m + 7, 1, 100)
    on = _session_run(p, stops, every, fused, batch)
    off = _session_run(p, stops, 0, fused, batch)
    assert len(on) == len(off)
    moved_out = False
    for (st1, k1, T1, d1, b1, a1), (st0, k0, T0, d0, b0, a0) in zip(on, off):
        T, d, base, done = _oracle_after(p, k1)
        assert k1 == k0 == done and st1 == st0
        assert same(T1, T) and same(d1, d) and np.array_equal(b1, base), k1
        assert same(T0, T) and np.array_equal(b0, base)
        assert a1 <= a0
        moved_out = moved_out or a1 < a0
    assert moved_out  # (basic slacks did leave the sweep)


@pytest.mark.parametrize("deact", [1, 8, 0])
@pytest.mark.parametrize("n,m,seed", [(300, 1100, 41100), (64, 128, 6528), (16, 1536, 1637), (129, 1513, 77)])
def test_deactivated_slacks_two_phase(gpu, n, m, seed, deact):
    p = sx.generateRandomProblem(n, m, seed, 1, 100)
    try:
        sx.set_deactivate(deact)
        got = sx.twoPhaseMethodEx(p)
    finally:
        sx.set_deactivate(sx.DEACTIVATE_EVERY)
    A, b, c = p.arrays()
    ref = two_phase_ref(A, b, c)
    assert got.status == ref["status"] and tuple(got.pivots) == ref["pivots"]
    assert np.array_equal(got.base, ref["base"])
    if got.status == sx.FEASIBLE:
        assert same(got.optimal_value, ref["opt"]) and same(got.solution, ref["x"])

