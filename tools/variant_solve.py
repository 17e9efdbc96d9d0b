"""Config 5's "degenerate" variant end to end: generateRandomProblem(8192, 32768, 851968, -100, 100)
(BASELINE.json configs[4]; the [-100, 100] range of main.cu:7-8 / randomInput main.cu:135-139), solved
by twoPhaseMethod on the GPU.  Records status, per-phase pivot counts, objective and time; for a
FEASIBLE answer checks a primal/dual certificate on the host from the final objective row
(simplex_last_objective_row: y_i = d[1+n+i], (A^T y - c)_j = d[1+j]):
  A x <= b, x >= 0, y >= 0, A^T y >= c (each within 1e-9 of the row's scale), |c.x - b.y| <= 1e-6 |c.x|.
For INFEASIBLE / DEGENERATE it records d[0] and the basic artificial variables
(twoPhaseMethod.cu:264-282).  (diagnostic; its output is the fixture tests/golden/variant_solves.json)
usage: python tools/variant_solve.py [n m seed lo hi] [--json out.json] [--limit PIVOTS] [--seconds S]
  --limit: phase-1 pivots before the instance is declared not to end (default 2,000,000);
  --seconds: also stop phase 1 after S seconds of pivoting (the record says which bound ended it);
  the record is rewritten after every chunk, so a run cut short still leaves its trace."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


CHUNK = 20000       # phase-1 pivots per progress line
P1_LIMIT = 2000000  # phase-1 pivots before the instance is declared not to end (no anti-cycling)


def certificate(A, b, c, x, d, n, m):
    """Primal/dual feasibility residuals scaled by each row's magnitude."""
    y = d[1 + n:1 + n + m]
    red = d[1:1 + n]
    Ax = A @ x
    Aty = A.T @ y
    scale_p = np.abs(A) @ np.abs(x) + np.abs(b) + 1.0
    scale_d = np.abs(A.T) @ np.abs(y) + np.abs(c) + 1.0
    cx, by = float(c @ x), float(b @ y)
    return {
        "primal_max_violation_rel": float(np.max((Ax - b) / scale_p)),
        "x_min": float(x.min()),
        "y_min": float(y.min()),
        "dual_max_violation_rel": float(np.max((c - Aty) / scale_d)),
        "reduced_cost_vs_Aty_minus_c_max_rel": float(np.max(np.abs(red - (Aty - c)) / scale_d)),
        "c_x": cx, "b_y": by, "gap_rel": abs(cx - by) / max(abs(cx), 1e-300),
        "basic_x": int(np.count_nonzero(x)),
    }


def main():
    argv = sys.argv[1:]
    opts = {}
    for k in ("--json", "--limit", "--seconds"):
        if k in argv:
            i = argv.index(k)
            opts[k] = argv[i + 1]
            del argv[i:i + 2]
    args = [a for a in argv if not a.startswith("--")]
    out_json = opts.get("--json")
    p1_limit = int(opts.get("--limit", P1_LIMIT))
    p1_seconds = float(opts.get("--seconds", 0)) or None
    n, m, seed, lo, hi = (int(a) for a in args) if args else (8192, 32768, 851968, -100, 100)
    import threading
    t_start = time.perf_counter()
    alive = threading.Event()

    def heartbeat():  # (a long solve prints nothing else: the GPU box's silence watchdog)
        while not alive.wait(30.0):
            print(f"  ... {time.perf_counter() - t_start:.0f} s", flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    import torch
    torch.cuda.set_device(0)
    import simplexoncuda_amd as sx
    # phase 1 alone first, in chunks (the reference has no iteration cap and no anti-cycling,
    # a cycling instance would never return), printing the phase-1 objective d[0]
    trace = []
    sess = sx.Session(generated=(n, m, seed, lo, hi))
    t1 = time.perf_counter()
    p1_status, p1_pivots = sx.NOT_ENDED, 0
    bound = "pivot_limit"
    neg = None

    def record(status):
        return {"instance": f"generateRandomProblem({n}, {m}, {seed}, {lo}, {hi})", "n": n, "m": m, "seed": seed,
                "lo": lo, "hi": hi, "status": status, "pivot_limit": p1_limit, "seconds_limit": p1_seconds,
                "ended_by": bound, "phase1_seconds": time.perf_counter() - t1, "phase1_trace": trace,
                "negated_rows": neg}

    while p1_pivots < p1_limit:
        tm = sess.pivots(CHUNK)
        p1_pivots = sess.total_pivots()
        p1_status = tm.status
        trace.append([int(p1_pivots), float(sess.objective())])
        print(f"  phase 1: {p1_pivots} pivots, d[0] = {trace[-1][1]:.9g}, status {p1_status}, "
              f"{time.perf_counter() - t1:.1f} s", flush=True)
        if p1_status != sx.NOT_ENDED:
            break
        if out_json and len(trace) % 10 == 0:
            with open(out_json, "w") as f:
                json.dump(record("PHASE1_RUNNING"), f, indent=1)
        if p1_seconds is not None and time.perf_counter() - t1 > p1_seconds:
            bound = "seconds_limit"
            break
    sess.close()
    prob = sx.generateRandomProblemDevice(n, m, seed, lo, hi)
    A, b, c = prob.arrays()
    neg = int(np.count_nonzero(b < -1e-9))
    if p1_status == sx.NOT_ENDED:
        alive.set()
        rec = record("PHASE1_NOT_ENDED")
        print(json.dumps(rec), flush=True)
        if out_json:
            with open(out_json, "w") as f:
                json.dump(rec, f, indent=1)
        return
    t0 = time.perf_counter()
    res = sx.twoPhaseMethodEx(prob, max_pivots=4 * max(p1_limit, p1_pivots))
    dt = time.perf_counter() - t0
    ph = sx.load()
    import ctypes
    sec = (ctypes.c_double * 2)()
    ph.simplex_last_phase_seconds(sec)
    d = sx.last_objective_row()
    rec = {"instance": f"generateRandomProblem({n}, {m}, {seed}, {lo}, {hi})", "n": n, "m": m, "seed": seed,
           "lo": lo, "hi": hi, "status": sx.STATUS_NAMES.get(res.status, res.status), "status_code": res.status,
           "pivots": list(res.pivots), "seconds": dt, "pivot_loop_s": [sec[0], sec[1]],
           "negated_rows": int(np.count_nonzero(b < -1e-9)), "phase1_trace": trace,
           "d0": float(d[0]) if len(d) else None,
           "d0_hex": float(d[0]).hex() if len(d) else None}
    if res.status == sx.FEASIBLE:
        rec["objective"] = res.optimal_value
        rec["objective_hex"] = float(res.optimal_value).hex()
        rec["certificate"] = certificate(A, b, c, res.solution, d, n, m)
    else:
        art = [int(i) for i in np.nonzero((res.base >= n + m) & (res.base < n + 2 * m))[0]]
        rec["basic_artificial_rows"] = art[:64]
        rec["basic_artificials"] = len(art)
    import hashlib
    rec["base_sha256"] = hashlib.sha256(np.ascontiguousarray(res.base, dtype=np.int32).tobytes()).hexdigest()
    alive.set()
    print(json.dumps(rec), flush=True)
    if out_json:
        with open(out_json, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
