"""Long oracle pins of config 5's [-100, 100] variant (SURVEY.md §8d's "degenerate" case,
main.cu:7-8 range): the CPU oracle's phase-1 state after 100, 250, 500
and 1000 pivots, made in the build container (the GPU box only reads the JSON).

  config5_degenerate  generateRandomProblem(8192, 32768, 851968, -100, 100)

The phase-1 tableau is built and canonicalised (twoPhaseMethod.cu:145-200, gaussian.cu:132-162)
and pivoted (solver.cu:78-126) by the serial restatement; only its row update runs on several
host threads (orc_set_threads: each element still receives exactly one operation, so the digests
do not depend on the thread count).  Stored per checkpoint: status, pivots, d[0], SHA-256 of the
bits of the logical tableau T (m x (1+n+2m) fp64, row-major), of d and of base, plus the
(entering, leaving) pair of every pivot up to the last checkpoint.

usage: python tests/golden/scripts/make_long_pins.py [threads]   (~25 GB RAM; hours)
"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import ctypes  # noqa: E402

import numpy as np  # noqa: E402

import oracle  # noqa: E402

CHECKPOINTS = [48, 100, 250, 500, 1000, 2000, 3000]  # 48: cross-checked against large_pivots.json
CASE = ("config5_degenerate", (8192, 32768, 851968, -100, 100))
OUT = os.path.join(ROOT, "tests", "golden", "long_pivots.json")


def sha(a):
    h = hashlib.sha256()
    mv = memoryview(np.ascontiguousarray(a)).cast("B")
    step = 1 << 28
    for k in range(0, len(mv), step):
        h.update(mv[k:k + step])
    return h.hexdigest()


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    lib = oracle.load()
    lib.orc_set_threads(threads)
    name, (n, m, seed, lo, hi) = CASE
    t0 = time.time()
    A, b, _ = oracle.generate(n, m, seed, lo, hi)
    T, d, base = oracle.build_phase1(A, b)
    del A
    oracle.update_objective(T, d, base)
    N = T.shape[1]
    print(f"built in {time.time() - t0:.1f}s", flush=True)
    rec = {"n": n, "m": m, "seed": seed, "lo": lo, "hi": hi, "width": int(N), "checkpoints": [], "pivot_er": []}
    e = ctypes.c_int64()
    r = ctypes.c_int64()
    k = 0
    st = oracle.NOT_ENDED
    t1 = time.time()
    for cp in CHECKPOINTS:
        while k < cp:
            st = lib.orc_pivot(oracle.p(T), m, N, T.strides[0] // 8, oracle.p(d), oracle.ip(base),
                               ctypes.byref(e), ctypes.byref(r))
            if st != oracle.NOT_ENDED:
                break
            rec["pivot_er"].append([int(e.value), int(r.value)])
            k += 1
        status = st if st != oracle.NOT_ENDED else oracle.PIVOT_CAP
        rec["checkpoints"].append({"pivots": k, "status": status, "d0": float(d[0]), "d0_hex": float(d[0]).hex(),
                                   "sha256_T": sha(T), "sha256_d": sha(d), "sha256_base": sha(base),
                                   "oracle_seconds": round(time.time() - t1, 1)})
        print(name, rec["checkpoints"][-1], flush=True)
        if k == 48:  # the threaded update reproduces the serial run's 48-pivot pin
            with open(os.path.join(ROOT, "tests", "golden", "large_pivots.json")) as f:
                old = json.load(f)[name]
            for key in ("sha256_T", "sha256_d", "sha256_base"):
                assert rec["checkpoints"][-1][key] == old[key], key
        with open(OUT, "w") as f:
            json.dump({name: rec}, f, indent=1, sort_keys=True)
        if st != oracle.NOT_ENDED:
            break


if __name__ == "__main__":
    main()
