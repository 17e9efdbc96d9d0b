"""A/B the sweep settings inside the real pivot loop (interleaved rounds, one process).

usage: python tools/sweep_update.py [config] [pivots_per_round] [rounds]
Prints, per (pivots per sweep, rows per step, sc1, waves) setting, the median pivots/s and the
sweep kernel's time and algorithmic GB/s.  Env SWEEP_BATCH / SWEEP_RB / SWEEP_SC1 / SWEEP_WAVES
(comma lists) choose the grid.
"""
import itertools
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (CONFIGS)


def _list(name, default, conv):
    return [conv(x) for x in os.environ.get(name, default).split(",")]


def main():
    import torch

    torch.cuda.set_device(0)
    import simplexoncuda_amd as sx

    cfg = sys.argv[1] if len(sys.argv) > 1 else "config3"
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 320
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    n, m, seed = bench.CONFIGS[cfg]
    s = sx.Session(generated=(n, m, seed, 1, 100))
    s.pivots(20)
    settings = list(itertools.product(_list("SWEEP_BATCH", "8,16,32", int), _list("SWEEP_RB", "1,2,4", int),
                                      _list("SWEEP_SC1", "0,1", int), _list("SWEEP_WAVES", "1", float)))
    res = {x: [] for x in settings}
    t = None
    for _ in range(rounds):
        for bt, rb, sc, wv in settings:
            sx.set_batch(bt)
            sx.set_update_rows(rb)
            sx.set_store_sc1(sc)
            sx.set_update_waves(wv)
            t = s.pivots(k, time_updates=1)
            res[(bt, rb, sc, wv)].append((t.pivots / t.wall_ms * 1e3, t.update_ms / max(t.update_launches, 1) * 1e3,
                                          t.swept_bytes / max(t.update_ms, 1e-9) / 1e6))
    for f, v in ((sx.set_batch, 0), (sx.set_update_rows, 0), (sx.set_store_sc1, -1), (sx.set_update_waves, 0)):
        f(v)
    print(f"{cfg}: {k} pivots x {rounds} rounds, stored width {t.stored_width}, swept bytes/sweep (last round) "
          f"{t.swept_bytes / max(t.update_launches, 1) / 1e9:.3f} GB; final status {t.status}")
    # settings run in a fixed order inside each round, so with slack compaction the later ones
    # sweep more active columns: compare the GB/s column, not the sweep time
    print("ranked by pivots/s; with slack compaction compare the GB/s column (later settings of a round "
          "sweep more columns)")
    for key in sorted(res, key=lambda x: -statistics.median(r[0] for r in res[x])):
        pv = statistics.median(r[0] for r in res[key])
        up = statistics.median(r[1] for r in res[key])
        gb = statistics.median(r[2] for r in res[key])
        print(f"batch={key[0]:2d} rb={key[1]} sc1={key[2]} waves={key[3]}: {pv:9.1f} pivots/s  sweep {up:8.1f} us  "
              f"{gb:7.1f} GB/s")


if __name__ == "__main__":
    main()
