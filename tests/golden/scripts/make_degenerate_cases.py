"""LPs whose two-phase solve ends DEGENERATE (-3): phase 1 reaches zero infeasibility with an
artificial variable still basic (twoPhaseMethod.cu:206-223, 270-282), so phase 2 is skipped.
Generated instances of generateRandomProblem essentially never do (continuous data); these
are small integer LPs with redundant rows, found by the CPU oracle, plus larger instances that
embed each of them block-diagonally next to a generated [1,100] instance (hundreds to
thousands of phase-1 pivots over several 512-row tiles).  Run in the build container; the
GPU tests read tests/golden/degenerate_cases.json.

usage: python tests/golden/scripts/make_degenerate_cases.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import oracle  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "degenerate_cases.json")
EMBED = [(200, 300, 1), (300, 1100, 41100), (256, 1500, 5), (1000, 700, 9)]


def embed(big, small):
    """block-diagonal [[A_big, 0], [0, A_small]] with b, c stacked"""
    nb, mb, seed = big
    Ab, bb, cb = oracle.generate(nb, mb, seed, 1, 100)
    As, bs, cs = (np.array(x, dtype=np.float64) for x in small)
    ms, ns = As.shape
    A = np.zeros((mb + ms, nb + ns))
    A[:mb, :nb] = Ab
    A[mb:, nb:] = As
    return A, np.concatenate([bb, bs]), np.concatenate([cb, cs])


def main():
    rng = np.random.default_rng(1)
    small = []
    while len(small) < 4:
        n, m = int(rng.integers(2, 6)), int(rng.integers(2, 6))
        A = rng.integers(-3, 4, size=(m, n)).astype(float)
        b = rng.integers(-3, 4, size=m).astype(float)
        c = rng.integers(-3, 4, size=n).astype(float)
        if rng.random() < 0.5:
            k, j = int(rng.integers(0, m)), int(rng.integers(0, m))
            A[j], b[j] = A[k], b[k]
        r = oracle.two_phase(A, b, c)
        if r["status"] == oracle.DEGENERATE:
            small.append({"A": A.tolist(), "b": b.tolist(), "c": c.tolist(), "status": r["status"],
                          "pivots": list(r["pivots"]), "base": r["base"].tolist()})
    large = []
    for k, big in enumerate(EMBED):
        s = small[k % len(small)]
        A, b, c = embed(big, (s["A"], s["b"], s["c"]))
        r = oracle.two_phase(A, b, c, max_pivots=50000)
        assert r["status"] == oracle.DEGENERATE, r["status"]
        large.append({"big": list(big), "small": k % len(small), "status": r["status"],
                      "pivots": list(r["pivots"]), "base": r["base"].tolist()})
    with open(OUT, "w") as f:
        json.dump({"small": small, "embedded": large}, f)
    print(len(small), "small,", len(large), "embedded:", [x["pivots"] for x in large])


if __name__ == "__main__":
    main()
