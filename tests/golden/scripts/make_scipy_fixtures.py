"""Independent LP optima (SciPy / HiGHS) for small generated instances -> scipy_optima.json.

Run in the build container only (SciPy is not needed on the GPU box).  The instances are
produced by the oracle's restatement of generateRandomProblem (problem.cu:49-126), so the
fixture pins the oracle's simplex to an independent solver on the same data.
"""
import json
import os
import sys

import numpy as np
from scipy.optimize import linprog

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "..", "oracle"))
import oracle  # noqa: E402

CASES = [
    # (n, m, seed, lo, hi)
    (20, 10, 2010, 1, 100),      # config 1 generated instance (seed n*100+m, main.cu:63)
    (3, 2, 302, 1, 100),
    (30, 40, 3040, 1, 100),
    (64, 64, 6464, 1, 100),
    (128, 64, 12864, 1, 100),
    (64, 128, 6528, 1, 100),
    (256, 256, 25856, 1, 100),   # smallest published -t instance
    (20, 10, 2010, -100, 100),   # default CLI range (main.cu:7-8): mixed-sign b
    (8, 6, 7, -100, 100),
    (40, 30, 4030, -100, 100),
    (25, 25, 99, -100, 100),
]


def main():
    out = []
    for n, m, seed, lo, hi in CASES:
        A, b, c = oracle.generate(n, m, seed, lo, hi)
        r = linprog(-c, A_ub=A, b_ub=b, bounds=[(0, None)] * n, method="highs")
        rec = {"n": n, "m": m, "seed": seed, "lo": lo, "hi": hi, "highs_status": int(r.status)}
        if r.status == 0:
            rec["highs_opt"] = float(-r.fun)
        out.append(rec)
        print(rec, file=sys.stderr)
    with open(os.path.join(HERE, "..", "scipy_optima.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
