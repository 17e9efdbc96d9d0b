"""A/B of sweep settings on synthetic matrices through simplex_bench_sweep (diagnostic):
32 pending pivots, per size, for each variant "sc1:rows:stages[:cols[:oop]]" (write-through stores,
rows per step, LDS-DMA stages per wave -- 0 = the register sweep, columns per thread -- 2 =
k_sweep, 1 = k_sweep1, out of place -- 1 = read one buffer and write another).
usage: python tools/sweep_bench_ab.py [rowsxcols ...] [variants=1:4:0,1:4:3,...] [ld_pad=0,31744]
(default sizes: the config-3' 4096x8192 and a few sizes around the 256 MB Infinity Cache)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    torch.cuda.set_device(0)
    import simplexoncuda_amd as sx
    lib = sx.load()
    args = [a for a in sys.argv[1:] if "=" not in a]
    opts = dict(a.split("=", 1) for a in sys.argv[1:] if "=" in a)
    sizes = [tuple(int(v) for v in a.split("x")) for a in args] or \
        [(1024, 4096), (2048, 8192), (3072, 8192), (4096, 8192), (8192, 8192)]
    variants = [tuple(int(x) for x in v.split(":"))
                for v in opts.get("variants", "0:2:0,0:4:0,1:2:0,1:4:0").split(",")]
    pads = [int(x) for x in opts.get("ld_pad", "0").split(",")]
    for rnd in range(2):
        for (rows, cols), pad in ((sz, p) for sz in sizes for p in pads):
            lib.simplex_set_ld_pad(pad)
            for v in variants:
                sc1, rb, d = v[:3]
                cpt = v[3] if len(v) > 3 else 2  # columns per thread
                oop = v[4] if len(v) > 4 else 0
                lib.simplex_set_sweep_cols(cpt)
                lib.simplex_set_sweep_oop(oop)
                lib.simplex_set_store_sc1(sc1)
                lib.simplex_set_update_rows(rb)
                lib.simplex_set_sweep_stages(d)
                us, nbytes = sx.bench_sweep(rows, cols, 823296, 1, 100, 32, warmup=5, iters=50)
                print(f"round {rnd} {rows}x{cols} ({8 * rows * cols / 2**20:5.0f} MiB) ld_pad={pad} sc1={sc1} "
                      f"rows={rb} stages={d} cols={cpt} oop={oop}: {us:7.1f} us {nbytes / us / 1e3:6.0f} GB/s "
                      f"frac {nbytes / us / 1e3 / 8000:.3f}", flush=True)
    lib.simplex_set_store_sc1(-1)
    lib.simplex_set_update_rows(0)
    lib.simplex_set_sweep_stages(0)
    lib.simplex_set_sweep_cols(2)
    lib.simplex_set_sweep_oop(0)
    lib.simplex_set_ld_pad(0)


if __name__ == "__main__":
    main()
