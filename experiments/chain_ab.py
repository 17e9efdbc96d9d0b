"""A/B of fused-batch settings in the real pivot loop (diagnostic): for each setting and config,
W untimed + K timed phase-1 pivots; per pivot: wall time, sweep time (HIP events) and the rest
(the chain: the fused batch + slack exchanges), plus the in-kernel stamp breakdown of one batch.

usage: python tools/chain_ab.py <setting>=<v1>,<v2> [config=config5,config3] [rounds=2]
  settings: regions (simplex_set_regions: 0 plain rows, 1 two-region layout),
            rows (simplex_set_update_rows: rows per sweep step, 0 = auto),
            waves (simplex_set_update_waves: the sweep's grid as a multiple of the resident blocks),
            policy (simplex_set_store_sc1: the sweep's cache policy 0..4, -1 = default),
            mfma (simplex_set_sweep_mfma: 0 vector sweep, 1 matrix-core sweep, -1 auto),
            shadow (simplex_set_shadow_sweep: 0 off, -1 / cap: a concurrent shadow sweep per batch),
            batch (simplex_set_batch: pivots per batch and sweep, 0 = default)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

PIVOTS = {"config5": 640, "config4": 1280, "config3": 3200, "config2": 1600}  # (timed, after 128)


def stamps_summary(s, k=32, nb=6):
    rows = []
    for _ in range(nb):
        st = s.stamps(k)
        if st is None:
            return None
        st = st.astype(np.int64)
        for q in range(k - 1):
            a, nxt = st[q], st[q + 1, 0]
            rows.append([a[2] - a[0], a[1] - a[2], a[3] - a[1], a[6] - a[3], a[7] - a[6], a[4] - a[7], a[5] - a[4],
                         nxt - a[5], nxt - a[0]])
    return np.median(np.array(rows) * 0.01, axis=0)


def main():
    import torch
    torch.cuda.set_device(0)
    import simplexoncuda_amd as sx
    lib = sx.load()
    args = dict(a.split("=", 1) for a in sys.argv[1:])
    configs = args.pop("config", "config5,config3").split(",")
    rounds = int(args.pop("rounds", "2"))
    (name, vals), = args.items()
    setter = {"regions": lambda v: lib.simplex_set_regions(int(v)),
              "rows": lambda v: lib.simplex_set_update_rows(int(v)),
              "waves": lambda v: lib.simplex_set_update_waves(float(v)),
              "policy": lambda v: lib.simplex_set_store_sc1(int(v)),
              "mfma": lambda v: lib.simplex_set_sweep_mfma(int(v)),
              "shadow": lambda v: lib.simplex_set_shadow_sweep(int(v)),
              "batch": lambda v: lib.simplex_set_batch(int(v))}[name]
    reset = {"regions": 1, "rows": 0, "waves": 0, "policy": -1, "mfma": -1, "shadow": 0, "batch": 0}[name]
    print("stamps (us): ratio compute | ratio argmin+publish | -> selection seen | pass2 + row details |"
          " row compute | obj argmin+publish | -> entering seen | entering history | pivot")
    for r in range(rounds):
        for cfg in configs:
            n, m, seed = bench.CONFIGS[cfg]
            for v in vals.split(","):
                setter(v)
                s = sx.Session(generated=(n, m, seed, 1, 100))
                s.pivots(128)
                tim = s.pivots(PIVOTS[cfg] // s.batch() * s.batch(), time_updates=1)
                st = stamps_summary(s)
                s.close()
                per = tim.wall_ms * 1e3 / tim.pivots
                sw = tim.update_ms * 1e3 / tim.pivots
                print(f"round {r} {cfg} {name}={v}: {1e6 / per:8.0f} pivots/s  {per:6.2f} us/pivot = sweep {sw:5.2f}"
                      f" + rest {per - sw:5.2f}  | stamps " + (" ".join(f"{x:5.2f}" for x in st) if st is not None
                                                             else "-"), flush=True)
    setter(reset)


if __name__ == "__main__":
    main()
