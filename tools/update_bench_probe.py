"""The update kernel alone on synthetic matrices of several sizes (bench.py update_bench's
measurement, SURVEY.md §8d config 3'), for rocprofv3 --pmc passes per size: north_star's 4096 x 8192
(268 MB, about the 256 MB Infinity Cache) and larger ones that cannot stay in it.  (diagnostic)
usage: python tools/update_bench_probe.py rows cols [pivots ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rows, cols = int(sys.argv[1]), int(sys.argv[2])
    pivots = [int(a) for a in sys.argv[3:]] or [32, 64]
    import torch
    torch.cuda.set_device(0)
    import simplexoncuda_amd as sx
    for k in pivots:
        runs = [sx.bench_sweep(rows, cols, 823296, 1, 100, k, warmup=10, iters=50) for _ in range(3)]
        us, nbytes = sorted(runs)[1]
        print(f"{rows}x{cols} pivots {k}: median {us:.1f} us/sweep ({[round(r[0], 1) for r in runs]}), "
              f"{nbytes / 1e6:.1f} MB/sweep, {nbytes / us / 1e3:.0f} GB/s = {nbytes / us / 1e3 / 8000:.3f} of 8 TB/s, "
              f"{us / k:.2f} us/pivot", flush=True)


if __name__ == "__main__":
    main()
