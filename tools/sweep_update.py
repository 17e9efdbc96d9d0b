"""A/B the update-kernel settings inside the real pivot loop (interleaved rounds, one process).

usage: python tools/sweep_update.py [config] [pivots_per_round] [rounds]
Prints, per (rows/block, snake, sc1) setting, the median pivots/s and update-kernel time.
"""
import itertools
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (CONFIGS)


def main():
    import torch

    torch.cuda.set_device(0)
    import simplexoncuda_amd as sx

    cfg = sys.argv[1] if len(sys.argv) > 1 else "config3"
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    n, m, seed = bench.CONFIGS[cfg]
    s = sx.Session(sx.generateRandomProblem(n, m, seed, 1, 100))
    s.pivots(20)
    settings = list(itertools.product([1, 2, 4], [0, 1], [0, 1]))
    res = {x: [] for x in settings}
    for _ in range(rounds):
        for rb, sn, sc in settings:
            sx.set_update_rows(rb)
            sx.set_snake(sn)
            sx.set_store_sc1(sc)
            t = s.pivots(k, time_updates=4)
            res[(rb, sn, sc)].append((t.pivots / t.wall_ms * 1e3, t.update_ms / t.update_launches * 1e3))
    print(f"{cfg}: {k} pivots x {rounds} rounds, stored width {t.stored_width}, bytes/launch {t.update_bytes/1e9:.3f} GB")
    for key in sorted(res, key=lambda x: -statistics.median(r[0] for r in res[x])):
        pv = statistics.median(r[0] for r in res[key])
        up = statistics.median(r[1] for r in res[key])
        print(f"rb={key[0]} snake={key[1]} sc1={key[2]}: {pv:9.1f} pivots/s  update {up:8.1f} us  "
              f"{t.update_bytes / up / 1e3:7.1f} GB/s")


if __name__ == "__main__":
    main()
