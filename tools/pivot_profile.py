"""Update-kernel time by pivot kind (diagnostic).  For every setting two fresh resident
sessions of the same instance run the same pivots back to back: one with every update timed
(per-launch log: rows swept, microseconds), one untimed for the pivot rate.  Pivots are split
into sparse ones (< 10 % of the rows have a nonzero entering-column entry -- mostly slack
columns entering) and dense ones.

usage: python tools/pivot_profile.py [--settings "mode,rb,snake,sc1,waves,skip;..."]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--m", type=int, default=4096)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--pivots", type=int, default=600)
    ap.add_argument("--settings", default="-1,0,-1,-1,1,1;1,0,-1,-1,1,1;1,0,-1,-1,1,0")
    ap.add_argument("--out", default="gpurun_out/pivot_profile.json")
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    import simplexoncuda_amd as sx
    n, m = args.n, args.m
    res = {}
    cls = None
    for spec in args.settings.split(";"):
        mode, rb, sn, sc, wv, skip = spec.split(",")
        sx.set_update_mode(int(mode))
        sx.set_update_rows(int(rb))
        sx.set_snake(int(sn))
        sx.set_store_sc1(int(sc))
        sx.set_update_waves(float(wv))
        sx.set_skip_zero(int(skip))
        s = sx.Session(generated=(n, m, n * 100 + m, 1, 100))
        s.pivots(args.warmup)
        s.pivots(args.pivots, time_updates=1)
        rows, us = s.launch_log()
        s.close()
        s = sx.Session(generated=(n, m, n * 100 + m, 1, 100))
        s.pivots(args.warmup)
        t = s.pivots(args.pivots)
        s.close()
        if cls is None and int(skip):
            cls = rows < m // 10
        c = cls if cls is not None else rows < m // 10
        res[spec] = {"rows": rows.tolist(), "us": us.tolist(), "wall_ms": t.wall_ms, "pivots": t.pivots}
        sp, de = us[c], us[~c]
        print(f"mode,rb,snake,sc1,waves,skip={spec:18s} sparse {len(sp):3d} upd {sp.mean() if len(sp) else 0:7.1f} us"
              f" | dense {len(de):3d} upd {de.mean() if len(de) else 0:7.1f} us | untimed "
              f"{t.pivots / t.wall_ms * 1e3:8.1f} pivots/s", flush=True)
    for f in (sx.set_update_mode, sx.set_update_rows, sx.set_snake, sx.set_store_sc1):
        f(-1 if f is not sx.set_update_rows else 0)
    sx.set_update_waves(0)
    sx.set_skip_zero(1)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
