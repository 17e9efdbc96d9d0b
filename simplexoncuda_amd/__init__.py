"""simplexoncuda_amd -- MI355X-native dense two-phase simplex (drop-in for rik1599/SimplexOnCuda).

The solver is libsimplex_hip.so: hand-written gfx950 HIP kernels behind the reference's C
host API (include/problem.h, tabular.h, solver.h, twoPhaseMethod.h).  This package is the
thin Python mirror of that API; see DESIGN.md.
"""
from .api import (  # noqa: F401
    DEGENERATE, FEASIBLE, HANG, INFEASIBLE, NOT_ENDED, NUMERIC_FAIL, PIVOT_CAP, RAND_GLIBC, RAND_MSVC,
    STATUS_NAMES, UNBOUNDED, Problem, Result, Session, bench_sweep, dev_argmin, dev_build_phase1,
    dev_build_phase1_generated, dev_pivots, dev_update_objective, generateRandomProblem, last_objective_row,
    generateRandomProblemDevice, gpus, p2p_ready, printProblemToStream, readProblemFromFile, readRandomProblemFromFile,
    DEACTIVATE_EVERY, set_alias, set_batch, set_compact, set_deactivate, set_exchange_mode, set_force_exchange, set_fused, set_mr_single_launch,
    set_blocked, set_fine_pivot_rows, set_gpus, set_p2p, set_regions, set_replicated_objective, set_sweep_mfma,
    set_update_waves, set_verbose, set_virtual_ranks,
    twoPhaseMethod, twoPhaseMethodEx)
from ._lib import LIB_PATH, load  # noqa: F401
