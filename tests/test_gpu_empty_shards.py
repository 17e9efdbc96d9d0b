"""Shards that own no rows, solved again and again in one process (needs an MI355X).

Round 4's bisect saw W = 8 virtual-shard solves of a 1,100-row instance diverge from one shard
when the pending pivot rows U were allocated uncached.  Round 5 re-ran it
(profiles/r05_uncached_u_bisect.txt): be1d656^/be1d656 rebuilt on one box still diverged, from the
process's second multi-shard solve on, at W = 8 (1,100 rows: shards 3..7 own no rows) and also at
W = 2 (shards of 1,024 and 76 rows: no empty shard; status -3 after 417 and 529 pivots), and
HEAD itself failed this file's uncached case before every non-plain U was pooled for the process
(pivots (1321, 63) instead of (1318, 79)).  With the pool (sx_engine.cpp g_special: no engine
frees a fine-grained or uncached allocation) these tests pass.  This file keeps the conditions --
repeated solves in one process, empty and non-empty shards, each U allocation mode -- in the
default GPU suite, with the pivot-row check on (simplex_set_check_pivot_rows: every shard's U
against shard 0's before every sweep, no mismatch allowed).
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
def test_empty_shards_repeated_solves(gpu, umode, p2p):
    n, m = 300, 1100  # 512-row blocks: W = 8 leaves shards 3..7 without rows
    A, b, c = oracle.generate(n, m, n * 100 + m, 1, 100)
    ref = two_phase_ref(A, b, c)
    lib = sx.load()
    lib.simplex_set_fine_pivot_rows({"plain": 0, "fine": 1, "uncached": 2}[umode])
    lib.simplex_set_check_pivot_rows(1)
    bad0 = lib.simplex_pivot_row_mismatches()
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
                assert lib.simplex_pivot_row_mismatches() == bad0, where
    finally:
        lib.simplex_set_check_pivot_rows(0)
        lib.simplex_set_fine_pivot_rows(-1)
        sx.set_p2p(-1)
