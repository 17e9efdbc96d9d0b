"""Golden pins for BASELINE.json configs 4 and 5, made by the CPU oracle in
the build container (run once; the GPU box only reads the JSON it writes):

  config4            generateRandomProblem(4096, 16384, 425984, 1, 100)
  config5            generateRandomProblem(8192, 32768, 851968, 1, 100)
  config5_degenerate generateRandomProblem(8192, 32768, 851968, -100, 100)  (main.cu:7-8 range)

For each: the phase-1 tableau built and canonicalised (twoPhaseMethod.cu:145-200, gaussian.cu:
132-162), then PIVOTS phase-1 pivots (solver.cu:78-126) -- a full 32-pivot batch and a partial
one on the GPU side.  Stored: SHA-256 of the bits of the logical tableau T (m x (1+n+2m) fp64,
row-major, textbook orientation), of d (1+n+2m fp64) and of base (m int32), plus the status,
pivot count and d[0].  The reference publishes nothing above m = 8192, so only the oracle
pins these sizes.

usage: python tests/golden/scripts/make_large_fixtures.py [name ...]   (~4 min, ~25 GB RAM)
"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import oracle  # noqa: E402

PIVOTS = 48
CASES = {
    "config4": (4096, 16384, 425984, 1, 100),
    "config5": (8192, 32768, 851968, 1, 100),
    "config5_degenerate": (8192, 32768, 851968, -100, 100),
}
OUT = os.path.join(ROOT, "tests", "golden", "large_pivots.json")


def sha(a):
    h = hashlib.sha256()
    mv = memoryview(np.ascontiguousarray(a)).cast("B")
    step = 1 << 28
    for k in range(0, len(mv), step):
        h.update(mv[k:k + step])
    return h.hexdigest()


def main():
    names = sys.argv[1:] or list(CASES)
    res = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            res = json.load(f)
    for name in names:
        n, m, seed, lo, hi = CASES[name]
        t0 = time.time()
        A, b, _ = oracle.generate(n, m, seed, lo, hi)
        T, d, base = oracle.build_phase1(A, b)
        del A
        oracle.update_objective(T, d, base)
        t1 = time.time()
        st, done = oracle.solve(T, d, base, max_pivots=PIVOTS)
        t2 = time.time()
        res[name] = {"n": n, "m": m, "seed": seed, "lo": lo, "hi": hi, "pivots": done, "status": st,
                     "d0": float(d[0]), "sha256_T": sha(T), "sha256_d": sha(d), "sha256_base": sha(base),
                     "width": int(T.shape[1]), "oracle_seconds": round(t2 - t1, 1)}
        print(name, res[name], f"build {t1 - t0:.1f}s", flush=True)
        del T, d, base
        with open(OUT, "w") as f:
            json.dump(res, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
