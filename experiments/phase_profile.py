"""Whole-phase-1 profile of a generated instance (diagnostic): per-sweep pivots applied and
sweep time over every phase-1 pivot, plus the untimed wall time of the same phase.

usage: python tools/phase_profile.py [config] [out.json]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (CONFIGS)


def main():
    import torch

    torch.cuda.set_device(0)
    import simplexoncuda_amd as sx

    cfg = sys.argv[1] if len(sys.argv) > 1 else "config3"
    out = sys.argv[2] if len(sys.argv) > 2 else f"gpurun_out/phase_profile_{cfg}.json"
    n, m, seed = bench.CONFIGS[cfg]
    s = sx.Session(generated=(n, m, seed, 1, 100))
    t = s.pivots(12000, time_updates=1)
    rows, us = s.launch_log()
    s.close()
    s = sx.Session(generated=(n, m, seed, 1, 100))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    t2 = s.pivots(12000)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    s.close()
    res = {"config": cfg, "pivots": int(t2.pivots), "status": int(t2.status), "wall_s": wall,
           "pivots_per_s": t2.pivots / wall, "sweeps": len(rows), "sweep_us_mean": float(us.mean()),
           "sweep_GBps": float(t.swept_bytes / (t.update_ms / 1e3) / 1e9) if t.update_ms else None,
           "sweep_share": float(t.update_ms / t.wall_ms), "applied": rows.tolist(), "us": us.tolist()}
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump(res, f)
    print(json.dumps({k: v for k, v in res.items() if k not in ("applied", "us")}))


if __name__ == "__main__":
    main()
