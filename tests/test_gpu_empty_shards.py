"""Shards that own no rows, solved again and again in one process (needs an MI355X).

Round 4's bisect saw W = 8 virtual-shard solves of a 1,100-row instance diverge from one shard
when the pending pivot rows U were allocated uncached.  Round 5 re-ran it: on
the current code it never diverges (uncached, fine-grained or plain U; per-pivot exchange or
peer-memory batches), while be1d656^/be1d656 rebuilt on the same box still did in 2 of 3
repetitions -- only from the process's second W = 8 solve on, and only on instances where
512-row blocks leave shards empty (1,100 rows at W = 8: shards 3..7 own no rows;
profiles/r05_uncached_u_bisect.txt).  This file keeps exactly those conditions -- empty shards,
repeated solves in one process, each U allocation mode -- in the default GPU suite.
Bar: bit-exact against the oracle's whole two-phase solve (solver.cu:78-149,
twoPhaseMethod.cu:385-435).
"""
import numpy as np
import pytest

import oracle
import simplexoncuda_amd as sx
from conftest import two_phase_ref

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


@pytest.mark.parametrize("p2p", [0, 1])
@pytest.mark.parametrize("umode", ["plain", "fine", "uncached"])
def test_empty_shards_repeated_solves(gpu, monkeypatch, umode, p2p):
    n, m = 300, 1100  # 512-row blocks: W = 8 leaves shards 3..7 without rows
    A, b, c = oracle.generate(n, m, n * 100 + m, 1, 100)
    ref = two_phase_ref(A, b, c)
    lib = sx.load()
    if umode == "uncached":  # (diagnostic allocation, sx_engine.cpp alloc_shard)
        monkeypatch.setenv("SIMPLEX_DIAG_UNCACHED_U", "1")
    lib.simplex_set_fine_pivot_rows(1 if umode == "fine" else 0)
    sx.set_p2p(p2p)
    try:
        for rep in range(3):
            for W in (2, 8):
                p = sx.Problem.from_arrays(A, b, c)
                sx.set_virtual_ranks(W)
                try:
                    got = sx.twoPhaseMethodEx(p, 30000)  # (a cap: a diverged solve may cycle)
                finally:
                    sx.set_virtual_ranks(1)
                    p.close()
                where = f"rep {rep} W={W}"
                assert got.status == ref["status"], where
                assert tuple(got.pivots) == ref["pivots"], where
                assert np.array_equal(got.base, ref["base"]), where
                assert np.array_equal(bits(got.optimal_value), bits(ref["opt"])), where
                assert np.array_equal(bits(got.solution), bits(ref["x"])), where
    finally:
        lib.simplex_set_fine_pivot_rows(-1)
        sx.set_p2p(-1)
