"""Whole two-phase solves of larger instances by the serial CPU oracle -> oracle_solves.json.

The GPU path is bit-faithful to the oracle, so a whole solve pins status, per-phase pivot
counts, the optimal objective's bits, the final basis and the solution vector (SHA-256 of their
bytes).  These instances take the oracle minutes to an hour on one core, so the fixtures are
made here, in the build container, and the GPU tests compare against them
(tests/test_gpu_published.py).  Instances: config 3 (the reference's 8192 x 4096 -t instance,
main.cu:56-73) and n = 1024, m = 8192 with seed 110592 -- the MX250's INFEASIBLE record
(data/measures/mx250_2/benchmark_1024_8192.txt, SURVEY.md "Hard parts") -- and 110593 (the
RTX record's seed after the +1 hack, main.cu:63).

usage: python tests/golden/scripts/make_oracle_solves.py [name ...]
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "..", "oracle"))
import oracle  # noqa: E402

OUT = os.path.join(HERE, "..", "oracle_solves.json")
CASES = {
    "config3": (8192, 4096, 823296, 1, 100),
    "n1024_m8192_s110592": (1024, 8192, 110592, 1, 100),
    "n1024_m8192_s110593": (1024, 8192, 110593, 1, 100),
}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    names = sys.argv[1:] or list(CASES)
    out = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            out = json.load(f)
    for name in names:
        n, m, seed, lo, hi = CASES[name]
        A, b, c = oracle.generate(n, m, seed, lo, hi)
        t0 = time.time()
        r = oracle.two_phase(A, b, c)
        dt = time.time() - t0
        rec = {"n": n, "m": m, "seed": seed, "lo": lo, "hi": hi, "status": int(r["status"]),
               "pivots": list(r["pivots"]), "phase1_value": r["phase1_value"],
               "phase1_value_hex": float(r["phase1_value"]).hex(), "seconds": round(dt, 1),
               "base_sha256": sha(np.asarray(r["base"], dtype=np.int32))}
        if r["status"] == 0:
            rec["opt"] = r["opt"]
            rec["opt_hex"] = float(r["opt"]).hex()
            rec["x_sha256"] = sha(np.asarray(r["x"], dtype=np.float64))
        out[name] = rec
        print(name, rec, flush=True)
        with open(OUT, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
