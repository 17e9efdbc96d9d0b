"""Every block's hand-off stamps of 64-pivot fused batches: how much of each hand-off is the
producers' skew (first to last tile published) and how much the hop itself (last tile
published -> the consumers' pass 2 done).  (diagnostic)
usage: python tools/block_stamps.py [config5,config3]"""
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
    configs = (sys.argv[1] if len(sys.argv) > 1 else "config5,config3").split(",")
    for cfg in configs:
        n, m, seed = bench.CONFIGS[cfg]
        s = sx.Session(generated=(n, m, seed, 1, 100))
        s.pivots(256)
        NA = (m + 511) // 512
        NB = (n + 2 * m + 511) // 512  # phase 1: logical columns n + m slacks + m artificials
        acc = {k: [] for k in ("ratio skew", "ratio->obj hop", "obj details", "obj compute+publish",
                               "obj skew", "obj->ratio hop", "ratio next start", "pivot")}
        for _ in range(4):
            st, blk = s.block_stamps(64, NA + NB)
            if st is None:
                print(cfg, "stamps unavailable")
                break
            b = blk.astype(np.int64)
            for q in range(1, 63):
                ra, ob = b[q, :NA], b[q, NA:]
                rpub = ra[:, 1]
                osel, odet, opub = ob[:, 0], ob[:, 1], ob[:, 2]
                acc["ratio skew"].append(rpub.max() - rpub.min())
                acc["ratio->obj hop"].append(np.median(osel) - rpub.max())
                acc["obj details"].append(np.median(odet - osel))
                acc["obj compute+publish"].append(np.median(opub - odet))
                acc["obj skew"].append(opub.max() - opub.min())
                acc["obj->ratio hop"].append(np.median(ra[:, 2]) - opub.max())
                acc["ratio next start"].append(np.median(b[q + 1, :NA, 0] - ra[:, 2]))
                acc["pivot"].append(np.median(b[q + 1, :NA, 0] - ra[:, 0]))
        s.close()
        print(f"{cfg} (NA {NA}, NB {NB}) us: " + " | ".join(f"{k} {np.median(v) * 0.01:5.2f}" for k, v in acc.items()),
              flush=True)


if __name__ == "__main__":
    main()
