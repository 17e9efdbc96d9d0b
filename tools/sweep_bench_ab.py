"""A/B of sweep settings on synthetic matrices through simplex_bench_sweep (diagnostic):
write-through (sc1) stores on/off and rows per step, 32 pending pivots, per size.
usage: python tools/sweep_bench_ab.py [rowsxcols ...]   (default: the config-3' 4096x8192 and
a few sizes around the 256 MB Infinity Cache)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    torch.cuda.set_device(0)
    import simplexoncuda_amd as sx
    lib = sx.load()
    sizes = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1:]] or \
        [(1024, 4096), (2048, 8192), (3072, 8192), (4096, 8192), (8192, 8192)]
    for rnd in range(2):
        for rows, cols in sizes:
            for sc1 in (0, 1):
                for rb in (2, 4):
                    lib.simplex_set_store_sc1(sc1)
                    lib.simplex_set_update_rows(rb)
                    us, nbytes = sx.bench_sweep(rows, cols, 823296, 1, 100, 32, warmup=5, iters=50)
                    print(f"round {rnd} {rows}x{cols} ({8 * rows * cols / 2**20:5.0f} MiB) sc1={sc1} rows={rb}: "
                          f"{us:7.1f} us {nbytes / us / 1e3:6.0f} GB/s frac {nbytes / us / 1e3 / 8000:.3f}", flush=True)
    lib.simplex_set_store_sc1(-1)
    lib.simplex_set_update_rows(0)


if __name__ == "__main__":
    main()
