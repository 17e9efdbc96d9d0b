"""A/B of the sweep kernels on synthetic matrices (simplex_bench_sweep, diagnostic): the vector
sweep at 32 pending pivots, the matrix-core sweep at 32 and 64, per size; microseconds per sweep,
fraction of 8 TB/s, and per pivot.  usage: python tools/sweep_kernels_ab.py [rowsxcols ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    torch.cuda.set_device(0)
    import simplexoncuda_amd as sx
    sizes = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1:]] or [(4096, 8192), (32768, 9216),
                                                                          (32768, 10001), (4096, 11000)]
    for rnd in range(2):
        for rows, cols in sizes:
            for piv, mf in ((32, 0), (32, 1), (64, 1)):
                sx.set_sweep_mfma(mf)
                us, nb = sx.bench_sweep(rows, cols, 823296, 1, 100, piv, warmup=10, iters=40)
                print(f"round {rnd} {rows}x{cols} pivots={piv} mfma={mf}: {us:8.1f} us  frac "
                      f"{nb / us / 1e3 / 8000:.3f}  {us / piv:6.2f} us/pivot", flush=True)
    sx.set_sweep_mfma(-1)


if __name__ == "__main__":
    main()
