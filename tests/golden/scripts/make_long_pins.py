"""Long oracle pins of the full-size configs (VERDICT round 4 item 5, round 5
item 1): the CPU oracle's state after chosen pivot counts -- and, where it finishes, the whole
two-phase solve -- made in the build container (the GPU box only reads the JSON).

  config5_degenerate  generateRandomProblem(8192, 32768, 851968, -100, 100)  pivots 48..3000
  config5             generateRandomProblem(8192, 32768, 851968, 1, 100)     pivots 48, 320, 1600, 2080
                      (bench.py's timed window: the driver's --warmup 5 --steps 20 is pivots 320..1600),
                      every 5000 after, toward the whole solve (as far as the build container's time allows)
  config4             generateRandomProblem(4096, 16384, 425984, 1, 100)     pivots 48..2080, every
                      5000 after, then the whole two-phase solve (status, pivot counts, objective
                      bits, basis and solution digests: twoPhaseMethod.cu:225-435, :370-383)

The phase-1 tableau is built and canonicalised (twoPhaseMethod.cu:145-200, gaussian.cu:132-162)
and pivoted (solver.cu:78-126) by the serial restatement; only its row update runs on several
host threads (orc_set_threads: each element still receives exactly one operation, so the digests
do not depend on the thread count).  Stored per checkpoint: phase, status, pivots, d[0], SHA-256 of
the bits of the logical tableau T (m x width fp64, row-major; width = 1+n+2m in phase 1, 1+n+m in
phase 2), of d and of base.  Phase 2 follows orc_two_phase (twoPhaseMethod.cu:285-356).

A run saves its state to $PIN_STATE_DIR (default /tmp) at every checkpoint and resumes from it.

usage: python tests/golden/scripts/make_long_pins.py <case> [threads]   (config 5: ~25 GB RAM)
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

CASES = {
    "config5_degenerate": ((8192, 32768, 851968, -100, 100), [48, 100, 250, 500, 1000, 2000, 3000], False),
    "config5": ((8192, 32768, 851968, 1, 100), [48, 320, 1600, 2080] + list(range(5000, 200001, 5000)), True),
    "config4": ((4096, 16384, 425984, 1, 100), [48, 320, 1600, 2080] + list(range(5000, 200001, 5000)), True),
}
OUT = os.path.join(ROOT, "tests", "golden", "long_pivots.json")
# (a long run may write its progress elsewhere -- PIN_OUT -- and be merged into OUT when it is done,
# so a working tree sent to the GPU meanwhile keeps the committed pins)
OUT = os.environ.get("PIN_OUT", OUT)
STATE = os.environ.get("PIN_STATE_DIR", "/tmp")


def sha(a):
    h = hashlib.sha256()
    mv = memoryview(np.ascontiguousarray(a)).cast("B")
    step = 1 << 28
    for k in range(0, len(mv), step):
        h.update(mv[k:k + step])
    return h.hexdigest()


def save_rec(name, rec):
    allrec = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            allrec = json.load(f)
    allrec[name] = rec
    tmp = OUT + ".tmp"
    with open(tmp, "w") as f:
        json.dump(allrec, f, indent=1, sort_keys=True)
    os.replace(tmp, OUT)


def save_state(name, T, d, base, k, phase, rec):
    path = os.path.join(STATE, f"pins_{name}.npz")
    np.savez(path + ".tmp.npz", T=T, d=d, base=base, k=np.int64(k), phase=np.int64(phase),
             rec=np.frombuffer(json.dumps(rec).encode(), dtype=np.uint8))
    os.replace(path + ".tmp.npz", path)


def load_state(name):
    path = os.path.join(STATE, f"pins_{name}.npz")
    if not os.path.exists(path):
        return None
    z = np.load(path)
    return (z["T"], z["d"], z["base"], int(z["k"]), int(z["phase"]), json.loads(bytes(z["rec"]).decode()))


def checkpoint(rec, phase, k, st, T, width, d, base, t1):
    c = {"phase": phase, "pivots": k, "status": st, "d0": float(d[0]), "d0_hex": float(d[0]).hex(),
         "sha256_T": sha(np.ascontiguousarray(T[:, :width])), "sha256_d": sha(d), "sha256_base": sha(base),
         "oracle_seconds": round(time.time() - t1, 1)}
    rec["checkpoints"].append(c)
    return c


def main():
    name = sys.argv[1]
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    (n, m, seed, lo, hi), cps, whole = CASES[name]
    lib = oracle.load()
    lib.orc_set_threads(threads)
    N1, N2 = 1 + n + 2 * m, 1 + n + m
    t0 = time.time()
    A, b, c = oracle.generate(n, m, seed, lo, hi)
    st0 = load_state(name)
    if st0 is None:
        T, d, base = oracle.build_phase1(A, b)
        oracle.update_objective(T, d, base)
        k, phase = 0, 1
        rec = {"n": n, "m": m, "seed": seed, "lo": lo, "hi": hi, "width": int(N1), "width2": int(N2),
               "checkpoints": [], "seconds_before_resume": 0.0}
    else:
        T, d, base, k, phase, rec = st0
        print(f"resumed at phase {phase}, pivot {k}", flush=True)
    del A
    print(f"built in {time.time() - t0:.1f}s", flush=True)
    e = ctypes.c_int64()
    r = ctypes.c_int64()
    t1 = time.time() - rec.get("seconds_before_resume", 0.0)
    ld = T.shape[1]

    def pivot_to(target, width):
        nonlocal k
        st = oracle.NOT_ENDED
        while k < target:
            st = lib.orc_pivot(oracle.p(T), m, width, ld, oracle.p(d), oracle.ip(base), ctypes.byref(e),
                               ctypes.byref(r))
            if st != oracle.NOT_ENDED:
                return st
            k += 1
        return st

    st = oracle.NOT_ENDED
    if phase == 1:
        for cp in cps:
            if cp <= k:
                continue
            st = pivot_to(cp, N1)
            ended = st != oracle.NOT_ENDED
            c1 = checkpoint(rec, 1, k, st if ended else oracle.PIVOT_CAP, T, N1, d, base, t1)
            print(name, c1, flush=True)
            if k == 48 and not ended:  # the threaded update reproduces the serial run's 48-pivot pin
                with open(os.path.join(ROOT, "tests", "golden", "large_pivots.json")) as f:
                    old = json.load(f)[name]
                for key in ("sha256_T", "sha256_d", "sha256_base"):
                    assert c1[key] == old[key], key
            rec["seconds_before_resume"] = time.time() - t1
            save_rec(name, rec)
            if whole and (ended or cp >= 5000):
                save_state(name, T, d, base, k, 1, rec)
            if ended or cp == cps[-1]:
                break
        if not whole:
            return
        if st != oracle.FEASIBLE:  # phase 1 did not end optimal (PIVOT_CAP / UNBOUNDED)
            return
        # phase-1 end (twoPhaseMethod.cu:258-282)
        p1 = k
        rec["phase1"] = {"status": st, "pivots": p1, "d0": float(d[0]), "d0_hex": float(d[0]).hex()}
        if abs(float(d[0])) >= 1e-9 and float(d[0]) < 0:  # compare(d[0], 0) < 0 (macro.h:28-42)
            rec["result"] = {"status": oracle.INFEASIBLE, "pivots": [p1, 0]}
            save_rec(name, rec)
            return
        degenerate = bool(np.any((base >= n + m) & (base < n + 2 * m)))
        if degenerate:
            rec["result"] = {"status": oracle.DEGENERATE, "pivots": [p1, 0]}
            save_rec(name, rec)
            return
        # phase 2 (twoPhaseMethod.cu:285-356): artificial columns dropped, d[1..n] = -c, slacks 0
        d2 = np.zeros(N2)
        d2[0] = d[0]
        d2[1:1 + n] = -c
        lib.orc_update_objective(oracle.p(T), m, N2, ld, oracle.ip(base), oracle.p(d2))
        d = d2
        rec["phase1_end_pivot"] = p1
        k, phase = 0, 2
        rec["seconds_before_resume"] = time.time() - t1
        save_rec(name, rec)
        save_state(name, T, d, base, k, 2, rec)
    # phase 2
    p1 = rec["phase1_end_pivot"]
    while True:
        target = k + 500
        st = pivot_to(target, N2)
        ended = st != oracle.NOT_ENDED
        if ended:
            break
        rec["seconds_before_resume"] = time.time() - t1
        print(name, "phase 2 at", k, flush=True)
    x = np.zeros(n)
    for i in range(m):
        if base[i] < n:
            x[base[i]] = T[i, 0]
    c2 = checkpoint(rec, 2, k, st, T, N2, d, base, t1)
    rec["result"] = {"status": st, "pivots": [p1, k], "opt": float(d[0]), "opt_hex": float(d[0]).hex(),
                     "sha256_base": sha(base), "sha256_x": sha(x)}
    rec["seconds_before_resume"] = time.time() - t1
    print(name, "done", rec["result"], c2, flush=True)
    save_rec(name, rec)


if __name__ == "__main__":
    main()
