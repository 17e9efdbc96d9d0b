"""Grid-size A/B of the matrix-core sweeps (simplex_set_update_waves: resident-grid multiple) on
synthetic matrices (diagnostic).  usage: python tools/msweep_waves_ab.py [rowsxcols ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    torch.cuda.set_device(0)
    import simplexoncuda_amd as sx
    lib = sx.load()
    sizes = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1:]] or [(4096, 8192), (32768, 9216)]
    sx.set_sweep_mfma(1)
    for rnd in range(2):
        for rows, cols in sizes:
            for piv in (32, 64):
                for w in (0.5, 0.667, 0.75, 0.875, 1.0, 1.25, 1.5, 2.0):
                    lib.simplex_set_update_waves(w)
                    us, nb = sx.bench_sweep(rows, cols, 823296, 1, 100, piv, warmup=10, iters=40)
                    print(f"round {rnd} {rows}x{cols} pivots={piv} waves={w}: {us:8.1f} us  frac "
                          f"{nb / us / 1e3 / 8000:.3f}", flush=True)
    lib.simplex_set_update_waves(1.0)
    sx.set_sweep_mfma(-1)


if __name__ == "__main__":
    main()
