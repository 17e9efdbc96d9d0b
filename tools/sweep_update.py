"""A/B the update-kernel settings inside the real pivot loop (interleaved rounds, one process).

usage: python tools/sweep_update.py [config] [pivots_per_round] [rounds]
Prints, per (rows/iteration, snake, sc1, waves) setting, the median pivots/s and update-kernel time.
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
    sx.set_skip_zero(int(os.environ.get("SWEEP_SKIP", "1")))  # 0: every pivot a full sweep
    s = sx.Session(generated=(n, m, seed, 1, 100))
    s.pivots(20)
    waves = [float(w) for w in os.environ.get("SWEEP_WAVES", "1,2").split(",")]
    settings = list(itertools.product([1, 2, 4], [0, 1], [0, 1], waves))
    res = {x: [] for x in settings}
    for _ in range(rounds):
        for rb, sn, sc, wv in settings:
            sx.set_update_rows(rb)
            sx.set_snake(sn)
            sx.set_store_sc1(sc)
            sx.set_update_waves(wv)
            t = s.pivots(k, time_updates=4)
            res[(rb, sn, sc, wv)].append((t.pivots / t.wall_ms * 1e3, t.update_ms / t.update_launches * 1e3,
                                          t.touched_bytes / t.update_ms / 1e6))
    print(f"{cfg}: {k} pivots x {rounds} rounds, stored width {t.stored_width}, dense bytes/launch "
          f"{t.update_bytes/1e9:.3f} GB; final status {t.status}")
    for key in sorted(res, key=lambda x: -statistics.median(r[0] for r in res[x])):
        pv = statistics.median(r[0] for r in res[key])
        up = statistics.median(r[1] for r in res[key])
        gb = statistics.median(r[2] for r in res[key])
        print(f"rb={key[0]} snake={key[1]} sc1={key[2]} waves={key[3]}: {pv:9.1f} pivots/s  update {up:8.1f} us  "
              f"{gb:7.1f} GB/s (touched rows)")


if __name__ == "__main__":
    main()
