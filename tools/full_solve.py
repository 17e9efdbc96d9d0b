"""One-off: whole twoPhaseMethod solves of the larger BASELINE configs on one GPU (problem
synthesised on the GPU, copied to the host, then the drop-in call), with per-phase pivot-loop
times.  usage: python tools/full_solve.py [config ...]"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (CONFIGS)


def main():
    import torch

    torch.cuda.set_device(0)
    import simplexoncuda_amd as sx

    for cfg in sys.argv[1:] or ["config4", "config5"]:
        n, m, seed = bench.CONFIGS[cfg]
        prob = sx.generateRandomProblemDevice(n, m, seed, 1, 100)
        t0 = time.perf_counter()
        res = sx.twoPhaseMethodEx(prob)
        dt = time.perf_counter() - t0
        prob.close()
        ph = (ctypes.c_double * 2)()
        sx.load().simplex_last_phase_seconds(ph)
        print(json.dumps({"config": cfg, "n": n, "m": m, "seed": seed, "status": sx.STATUS_NAMES.get(res.status),
                          "pivots": list(res.pivots), "objective": res.optimal_value, "seconds": dt,
                          "pivot_loop_s": [ph[0], ph[1]],
                          "pivots_per_s": [res.pivots[k] / ph[k] if ph[k] > 0 else None for k in (0, 1)]}),
              flush=True)


if __name__ == "__main__":
    main()
