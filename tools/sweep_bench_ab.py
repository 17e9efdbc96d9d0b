"""A/B of sweep settings on the synthetic config-3' matrix (4096 x 8192 fp64,
32 pending pivots) through simplex_bench_sweep (diagnostic).
usage: python tools/sweep_bench_ab.py [rows cols]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    torch.cuda.set_device(0)
    import simplexoncuda_amd as sx
    lib = sx.load()
    rows, cols = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (4096, 8192)
    for rnd in range(2):
        for sc1 in (-1, 0, 1):
            for rb in (0, 2, 4):
                for waves in (1.0, 2.0):
                    lib.simplex_set_store_sc1(sc1)
                    lib.simplex_set_update_rows(rb)
                    lib.simplex_set_update_waves(waves)
                    us, nbytes = sx.bench_sweep(rows, cols, 823296, 1, 100, 32, warmup=5, iters=50)
                    print(f"round {rnd} sc1={sc1:2d} rows={rb} waves={waves}: {us:7.1f} us  "
                          f"{nbytes / us / 1e3:6.0f} GB/s  frac {nbytes / us / 1e3 / 8000:.3f}", flush=True)
    lib.simplex_set_store_sc1(-1)
    lib.simplex_set_update_rows(0)
    lib.simplex_set_update_waves(1.0)


if __name__ == "__main__":
    main()
