"""The final objective row as a certificate (simplex_last_objective_row).

Phase 2 of the reference (twoPhaseMethod.cu:285-356) starts from d = (0, -c, 0) and every pivot
adds a multiple of a tableau row, so at the end d = (b.y, A^T y - c, y) with y_i = d[1+n+i], the
slack column's entry: y is the dual solution, d[1+j] the reduced costs, and d[0] = b.y the
optimal value (strong duality).  When phase 1 (costs on the artificials) ends with d[0] < 0, the
slack part y = d[1+n:1+n+m] of the phase-1 row is a Farkas certificate of infeasibility of
{A x <= b, x >= 0}: y >= 0, A^T y = d[1:1+n] >= 0 and b.y = d[0] < 0.  These identities are
checked here on the CPU oracle's final row (oracle.last_objective_row, the oracle's counterpart
of the library call), negated rows (b < 0) included; the GPU's row is compared with the oracle's
bit for bit in test_gpu_certificate.
"""
import numpy as np
import pytest

import oracle

CASES = [(20, 10, 2010, 1, 100), (25, 25, 99, -100, 100), (40, 60, 4060, 1, 100), (30, 50, 3050, -100, 100),
         (20, 40, 2040, -100, 100), (10, 30, 1030, -100, 100), (50, 80, 5080, -100, 100), (64, 128, 6528, 1, 100)]


@pytest.mark.parametrize("n,m,seed,lo,hi", CASES)
def test_objective_row_is_a_certificate(n, m, seed, lo, hi):
    A, b, c = oracle.generate(n, m, seed, lo, hi)
    r = oracle.two_phase(A, b, c)
    d = oracle.last_objective_row()
    y = d[1 + n:1 + n + m]
    scale = max(1.0, float(np.abs(A).max()) * float(np.abs(y).sum()))
    tol = 1e-9 * scale
    if r["status"] == 0:  # FEASIBLE
        assert len(d) == 1 + n + m
        assert np.abs(d[1:1 + n] - (A.T @ y - c)).max() <= tol  # reduced costs
        assert abs(d[0] - b @ y) <= tol and d[0] == r["opt"]    # strong duality
        assert y.min() >= -tol and d[1:1 + n].min() >= -tol    # dual feasible: the phase ended optimal
    elif r["status"] == -1:  # INFEASIBLE: a Farkas certificate
        assert len(d) == 1 + n + 2 * m
        assert y.min() >= -tol
        assert np.abs(d[1:1 + n] - A.T @ y).max() <= tol and d[1:1 + n].min() >= -tol
        assert abs(b @ y - d[0]) <= tol and d[0] < 0
    else:
        pytest.skip(f"status {r['status']}: no certificate")
