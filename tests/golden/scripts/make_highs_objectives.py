"""Independent optimal objectives (SciPy 1.15 / HiGHS) of the BASELINE configs -> highs_objectives.json.

north_star asks for the optimal objective of the GPU path to match within 1e-6 relative; the
reference publishes no objective values (only per-pivot timings), so an independent LP solver
pins them.  Run in the build container only (SciPy never goes to the GPU box); the instances are
the oracle's restatement of generateRandomProblem (problem.cu:49-126) with the -t seeds
n*100+m (main.cu:63) -- the same data the GPU generator produces bit for bit
(tests/test_gpu_generator.py).  Each instance gets a wall-clock limit; an instance HiGHS does not
finish is recorded with its status (the test skips it).

usage: python tests/golden/scripts/make_highs_objectives.py [name ...] [--time-limit S] [--method highs-ipm]
(a method other than the default is recorded under "<name>_<method>")
"""
import json
import os
import sys
import time

import numpy as np
from scipy.optimize import linprog

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "..", "oracle"))
import oracle  # noqa: E402

OUT = os.path.join(HERE, "..", "highs_objectives.json")
CASES = {
    # name: (n, m, seed, lo, hi)
    "config2": (2048, 1024, 205824, 1, 100),
    "config3": (8192, 4096, 823296, 1, 100),
    "config4": (4096, 16384, 425984, 1, 100),
    "config5": (8192, 32768, 851968, 1, 100),
    "config5_pm100": (8192, 32768, 851968, -100, 100),  # SURVEY.md §8d "degenerate" variant (main.cu:7-8)
    "n1024_m8192_s110592": (1024, 8192, 110592, 1, 100),  # the MX250's INFEASIBLE record (SURVEY.md "Hard parts")
}


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    limit = 3600.0
    if "--time-limit" in sys.argv:
        limit = float(sys.argv[sys.argv.index("--time-limit") + 1])
        args = [a for a in args if a != sys.argv[sys.argv.index("--time-limit") + 1]]
    method = "highs"
    if "--method" in sys.argv:
        method = sys.argv[sys.argv.index("--method") + 1]
        args = [a for a in args if a != method]
    names = args or list(CASES)
    out = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            out = json.load(f)
    for name in names:
        n, m, seed, lo, hi = CASES[name]
        A, b, c = oracle.generate(n, m, seed, lo, hi)
        t0 = time.time()
        r = linprog(-c, A_ub=A, b_ub=b, bounds=[(0, None)] * n, method=method,
                    options={"time_limit": limit, "presolve": True})
        dt = time.time() - t0
        del A
        rec = {"n": n, "m": m, "seed": seed, "lo": lo, "hi": hi, "highs_status": int(r.status),
               "highs_message": str(r.message), "seconds": round(dt, 1), "scipy": "1.15.3", "method": method}
        if r.status == 0:
            rec["highs_opt"] = float(-r.fun)
        out[name if method == "highs" else f"{name}_{method}"] = rec
        print(name, rec, flush=True)
        with open(OUT, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
