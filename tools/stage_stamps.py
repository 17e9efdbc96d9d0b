"""In-kernel hand-off stamps of 64-pivot (two-stage) fused batches: the per-pivot chain split
into its steps, first stage (pivots 0..31) vs second stage (32..63).  (diagnostic)
usage: python tools/stage_stamps.py [config5,config3]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

STEPS = ["ratio compute", "ratio argmin+publish", "-> selection seen", "pass2 + row details", "row compute",
         "obj argmin+publish", "-> entering seen", "entering history", "pivot"]


def main():
    import torch
    torch.cuda.set_device(0)
    import simplexoncuda_amd as sx
    configs = (sys.argv[1] if len(sys.argv) > 1 else "config5,config3").split(",")
    for cfg in configs:
        n, m, seed = bench.CONFIGS[cfg]
        s = sx.Session(generated=(n, m, seed, 1, 100))
        s.pivots(256)
        rows = {0: [], 1: []}
        for _ in range(6):
            st = s.stamps(64)
            if st is None:
                print(cfg, "stamps unavailable")
                break
            st = st.astype(np.int64)
            for q in range(63):
                a, nxt = st[q], st[q + 1, 0]
                rows[q >= 32].append([a[2] - a[0], a[1] - a[2], a[3] - a[1], a[6] - a[3], a[7] - a[6], a[4] - a[7],
                                      a[5] - a[4], nxt - a[5], nxt - a[0]])
        s.close()
        for stg in (0, 1):
            med = np.median(np.array(rows[stg]) * 0.01, axis=0)
            print(f"{cfg} stage {stg + 1}: " + " | ".join(f"{k} {v:5.2f}" for k, v in zip(STEPS, med)), flush=True)


if __name__ == "__main__":
    main()
