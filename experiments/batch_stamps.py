"""Where a fused batch spends its time (diagnostic): in-kernel timestamps of the hand-offs of
k_batch over a few batches of config 3, as microseconds per pivot step.

usage: python tools/batch_stamps.py [config] [batches] [k]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import torch
    torch.cuda.set_device(0)
    import simplexoncuda_amd as sx
    cfg = sys.argv[1] if len(sys.argv) > 1 else "config3"
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    n, m, seed = bench.CONFIGS[cfg]
    s = sx.Session(generated=(n, m, seed, 1, 100))
    s.pivots(200)
    rows = []
    for _ in range(nb):
        st = s.stamps(k).astype(np.int64)
        # per pivot q: [0] ratio block 0 starts (entering known) [1] its tile published
        # [3] objective block 0 knows the selection [4] its tile published [5] ratio block 0 knows
        # the next entering variable; next pivot's [0]
        for q in range(k - 1):
            a = st[q]
            nxt = st[q + 1, 0]
            rows.append([a[1] - a[0], a[3] - a[1], a[4] - a[3], a[5] - a[4], nxt - a[5], nxt - a[0]])
    r = np.array(rows) * 0.01  # ticks of 10 ns -> us
    names = ["ratio tile", "-> selection seen", "objective tile", "-> entering seen", "entering history read",
             "pivot total"]
    for i, nm in enumerate(names):
        print(f"{nm:26s} median {np.median(r[:, i]):6.2f} us  mean {r[:, i].mean():6.2f}")
    s.close()


if __name__ == "__main__":
    main()
