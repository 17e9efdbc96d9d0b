"""simplex_last_objective_row against the oracle's final objective row, bit for bit (the
certificate identities themselves are checked on the oracle's row in test_certificate.py)."""
import numpy as np
import pytest

import oracle
import simplexoncuda_amd as sx
from test_certificate import CASES

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,m,seed,lo,hi", CASES)
def test_last_objective_row_matches_oracle(gpu, n, m, seed, lo, hi):
    p = sx.generateRandomProblem(n, m, seed, lo, hi)
    got = sx.twoPhaseMethodEx(p)
    d_gpu = sx.last_objective_row()
    A, b, c = p.arrays()
    r = oracle.two_phase(A, b, c)
    d_ref = oracle.last_objective_row()
    assert got.status == r["status"]
    assert d_gpu.shape == d_ref.shape
    assert np.array_equal(d_gpu.view(np.uint64), d_ref.view(np.uint64))
