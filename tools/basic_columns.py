"""How much of each sweep moves basic columns (diagnostic).

A column basic in row i is the unit vector e_i wherever the residuals a_k - fl(a_k / p) p of its
entry (solver.cu:34-46) rounded to +0, and every later pivot row holds +0 in it until row i leaves,
so the sweep rewrites such a column unchanged while its factors are finite.  This counts, at
phase-1 checkpoints of a generated instance, the stored columns a sweep moves (1 + n + touched
slacks) and how many of them are basic (0-based variable indices in base, as the oracle's).
usage: python tools/basic_columns.py [config] [checkpoint,...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import simplexoncuda_amd as sx  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "config5"
    cps = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else \
        [320, 1600, 2080, 5000, 10000, 20000, 40000, 60000, 80000]
    n, m, seed = bench.CONFIGS[name][:3]
    width = 1 + n + 2 * m
    sx.set_deactivate(0)  # (what the sweep would move without moving basic slacks out)
    s = sx.Session(generated=(n, m, seed, 1, 100))
    for k in cps:
        t = s.pivots(k - s.total_pivots())
        _, base = s.objective_row_and_basis(m, width)
        nact = s.active_slacks()
        # base[i]: the basic variable of row i, 0-based over the columns after the RHS (structural
        # < n <= slack < n + m <= artificial; orc_build_phase1).  A basic slack has been pivoted in, so
        # its row has left once and its column is among the moved ones; a basic artificial aliases
        # the untouched slack column of its row (not moved).
        struct = int(np.count_nonzero(base < n))
        slack = int(np.count_nonzero((base >= n) & (base < n + m)))
        art = int(np.count_nonzero(base >= n + m))
        moved = 1 + n + nact
        basic_moved = struct + slack
        print(f"{name} pivots {s.total_pivots():6d} status {t.status:3d}: moved columns {moved:6d}, basic among them "
              f"{basic_moved:6d} ({basic_moved / moved:5.1%}; structural {struct}, slack {slack}), "
              f"artificial basic {art}", flush=True)
        if t.status != sx.NOT_ENDED:
            break
    s.close()
    sx.set_deactivate(sx.DEACTIVATE_EVERY)


if __name__ == "__main__":
    main()
