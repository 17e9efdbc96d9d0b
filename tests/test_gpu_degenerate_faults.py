"""DEGENERATE outcomes, fused-batch fault recovery and batch-id wrap-around, on the GPU,
bit for bit against the CPU oracle.

* DEGENERATE (-3): phase 1 ends feasible with an artificial variable still basic
  (twoPhaseMethod.cu:206-223, 270-282) -- small integer LPs and larger ones that embed them
  (tests/golden/degenerate_cases.json, tests/golden/scripts/make_degenerate_cases.py).
* SIMPLEX_HANG recovery: a fused batch forced to abort (test hook) is undone -- objective row
  restored, basis never written -- and re-run on the per-pivot path; results unchanged.
* Batch ids wrap at 2^15 (the granule tags keep 15 bits): tagged words are cleared first.
"""
import json
import os

import numpy as np
import pytest

import oracle
import simplexoncuda_amd as sx
from conftest import GOLDEN, two_phase_ref

pytestmark = pytest.mark.gpu

with open(os.path.join(GOLDEN, "degenerate_cases.json")) as _f:
    CASES = json.load(_f)


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


def solve_both(A, b, c):
    p = sx.Problem.from_arrays(A, b, c)
    try:
        got = sx.twoPhaseMethodEx(p)
    finally:
        p.close()
    ref = two_phase_ref(A, b, c)
    assert got.status == ref["status"]
    assert tuple(got.pivots) == ref["pivots"]
    assert np.array_equal(got.base, ref["base"])
    if got.status == sx.FEASIBLE:
        assert np.array_equal(bits(got.optimal_value), bits(ref["opt"]))
        assert np.array_equal(bits(got.solution), bits(ref["x"]))
    return got


def embedded(case):
    nb, mb, seed = case["big"]
    s = CASES["small"][case["small"]]
    Ab, bb, cb = oracle.generate(nb, mb, seed, 1, 100)
    As, bs, cs = (np.array(s[k], dtype=np.float64) for k in ("A", "b", "c"))
    ms, ns = As.shape
    A = np.zeros((mb + ms, nb + ns))
    A[:mb, :nb] = Ab
    A[mb:, nb:] = As
    return A, np.concatenate([bb, bs]), np.concatenate([cb, cs])


@pytest.mark.parametrize("k", range(4))
def test_degenerate_small(gpu, k):
    s = CASES["small"][k]
    got = solve_both(np.array(s["A"]), np.array(s["b"]), np.array(s["c"]))
    assert got.status == sx.DEGENERATE == s["status"]
    assert list(got.pivots) == s["pivots"] and got.base.tolist() == s["base"]


@pytest.mark.parametrize("k", range(4))
@pytest.mark.parametrize("fused", [-1, 0])
def test_degenerate_embedded(gpu, k, fused):
    case = CASES["embedded"][k]
    sx.set_fused(fused)
    try:
        got = solve_both(*embedded(case))
    finally:
        sx.set_fused(-1)
    assert got.status == sx.DEGENERATE
    assert list(got.pivots) == case["pivots"] and got.base.tolist() == case["base"]


def test_degenerate_public_entry(gpu):
    """twoPhaseMethod (the reference signature) returns DEGENERATE itself"""
    case = CASES["embedded"][0]
    A, b, c = embedded(case)
    p = sx.Problem.from_arrays(A, b, c)
    try:
        st, _, _ = sx.twoPhaseMethod(p)
    finally:
        p.close()
    assert st == sx.DEGENERATE


# ------------------------------------------------------------------ fused-batch aborts
@pytest.mark.parametrize("batch", [0, 64])
@pytest.mark.parametrize("inject", [0, 3, 30])
def test_hang_recovery_bit_exact(gpu, inject, batch):
    """config 2's instance (2003 + 69 pivots, published): the inject-th fused batch of the
    solve aborts; it is undone and re-run (a two-stage batch: two per-pivot stages), and the
    whole solve stays bit-exact"""
    lib = sx.load()
    p = sx.generateRandomProblem(2048, 1024, 205824, 1, 100)
    r0 = lib.simplex_hang_recoveries()
    lib.simplex_set_hang_inject(inject)
    sx.set_batch(batch)
    try:
        got = solve_both(*p.arrays())
    finally:
        sx.set_batch(0)
        lib.simplex_set_hang_inject(-1)
        p.close()
    assert lib.simplex_hang_recoveries() == r0 + 1
    assert tuple(got.pivots) == (2003, 69)


@pytest.mark.parametrize("batch,slot", [(0, 5), (0, 31), (64, 20), (64, 45)])
def test_hang_recovery_mid_batch(gpu, batch, slot):
    """the abort inside a running batch -- `slot` pivots already applied to the
    objective row (and, past slot 32, the second stage started) when ratio block 0 leaves and
    the other blocks time out.  The host restores d from d_save (each entry saved by the thread
    that wrote it) and re-runs the batch; the solve stays bit-exact"""
    lib = sx.load()
    p = sx.generateRandomProblem(2048, 1024, 205824, 1, 100)
    r0 = lib.simplex_hang_recoveries()
    lib.simplex_set_hang_inject(3)
    lib.simplex_set_hang_inject_slot(slot)
    sx.set_batch(batch)
    try:
        got = solve_both(*p.arrays())
    finally:
        sx.set_batch(0)
        lib.simplex_set_hang_inject(-1)
        lib.simplex_set_hang_inject_slot(-1)
        p.close()
    assert lib.simplex_hang_recoveries() == r0 + 1
    assert tuple(got.pivots) == (2003, 69)


@pytest.mark.parametrize("batch,slot", [(0, 9), (64, 40)])
def test_hang_recovery_mid_batch_multirank(gpu, batch, slot):
    """the same inside a peer-memory batch of 2 virtual shards: rank 0's ratio block 0 leaves at
    `slot` (64: in the second stage), its peers time out; every shard restores its own slice of
    d and re-runs the batch"""
    lib = sx.load()
    p = sx.generateRandomProblem(129, 1513, 77, -100, 100)
    r0 = lib.simplex_hang_recoveries()
    sx.set_virtual_ranks(2)
    sx.set_p2p(1)
    sx.set_batch(batch)
    lib.simplex_set_hang_inject(2)
    lib.simplex_set_hang_inject_slot(slot)
    try:
        solve_both(*p.arrays())
    finally:
        lib.simplex_set_hang_inject(-1)
        lib.simplex_set_hang_inject_slot(-1)
        sx.set_batch(0)
        sx.set_p2p(-1)
        sx.set_virtual_ranks(1)
        p.close()
    assert lib.simplex_hang_recoveries() == r0 + 1


def test_hang_recovery_twice_falls_back(gpu):
    """two aborts in one phase: the rest of the phase runs on the per-pivot path"""
    lib = sx.load()
    p = sx.generateRandomProblem(300, 1100, 41100, 1, 100)
    r0 = lib.simplex_hang_recoveries()
    try:
        for k in (2, 0):  # the 2nd fused batch, then the first one after the re-run
            lib.simplex_set_hang_inject(k)
            got = solve_both(*p.arrays())
    finally:
        lib.simplex_set_hang_inject(-1)
        p.close()
    assert lib.simplex_hang_recoveries() == r0 + 2
    assert got.status == sx.FEASIBLE


@pytest.mark.parametrize("W", [2, 3])
def test_hang_recovery_multirank(gpu, W):
    """virtual shards on the peer-memory fused batch: every shard aborts the same batch and
    all re-run it on the exchange path"""
    lib = sx.load()
    p = sx.generateRandomProblem(129, 1513, 77, -100, 100)
    r0 = lib.simplex_hang_recoveries()
    sx.set_virtual_ranks(W)
    sx.set_p2p(1)
    lib.simplex_set_hang_inject(2)
    try:
        solve_both(*p.arrays())
    finally:
        lib.simplex_set_hang_inject(-1)
        sx.set_p2p(-1)
        sx.set_virtual_ranks(1)
        p.close()
    assert lib.simplex_hang_recoveries() == r0 + 1


# ------------------------------------------------------------------ batch ids wrap
@pytest.mark.parametrize("mode", ["fused", "fused64", "unfused", "p2p2"])
def test_batch_id_wrap(gpu, mode):
    """the solve starts 20 batch ids before the wrap (ids 1..32767) and crosses it (fused64:
    two-stage batches, whose second-stage leaving slots live in PM2)"""
    lib = sx.load()
    p = sx.generateRandomProblem(2048, 1024, 205824, 1, 100)
    lib.simplex_set_first_batch_id(32767 - 20)
    if mode == "unfused":
        sx.set_fused(0)
    if mode == "fused64":
        sx.set_batch(64)
    if mode == "p2p2":
        sx.set_virtual_ranks(2)
        sx.set_p2p(1)
    try:
        got = solve_both(*p.arrays())
    finally:
        lib.simplex_set_first_batch_id(1)
        sx.set_batch(0)
        sx.set_fused(-1)
        sx.set_p2p(-1)
        sx.set_virtual_ranks(1)
        p.close()
    assert tuple(got.pivots) == (2003, 69)
