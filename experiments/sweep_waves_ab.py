"""A/B of the sweep's resident-grid size on synthetic matrices (simplex_bench_sweep, diagnostic):
for each size, rows per step, cache policy (simplex_set_store_sc1 0..4) and `waves` value (the
grid = waves x blocks resident on the device), the microseconds per 32-pivot sweep, 3 rounds
interleaved.
usage: python tools/sweep_waves_ab.py [rowsxcols ...] [waves=0.25,0.5,1] [rb=4] [pol=1] [mfma=0,1]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    torch.cuda.set_device(0)
    import simplexoncuda_amd as sx
    args = [a for a in sys.argv[1:] if "=" not in a]
    opts = dict(a.split("=", 1) for a in sys.argv[1:] if "=" in a)
    sizes = [tuple(int(v) for v in a.split("x")) for a in args] or [(4096, 8192)]
    waves = [float(w) for w in opts.get("waves", "0.25,0.5,0.75,1,2").split(",")]
    rbs = [int(r) for r in opts.get("rb", "4").split(",")]
    pols = [int(r) for r in opts.get("pol", "1").split(",")]
    mfmas = [int(r) for r in opts.get("mfma", "0").split(",")]
    for rnd in range(3):
        for rows, cols in sizes:
            for rb in rbs:
                sx.set_update_rows(rb)
                for pol in pols:
                    sx.set_store_sc1(pol)
                    for mf in mfmas:
                        sx.set_sweep_mfma(mf)
                        for w in waves:
                            sx.set_update_waves(w)
                            us, nbytes = sx.bench_sweep(rows, cols, 823296, 1, 100, 32, warmup=10, iters=50)
                            print(f"round {rnd} {rows}x{cols} rb={rb} pol={pol} mfma={mf} waves={w:g}: {us:7.1f} us "
                                  f"{nbytes / us / 1e3:6.0f} GB/s frac {nbytes / us / 1e3 / 8000:.3f}", flush=True)
    sx.set_update_waves(0)
    sx.set_update_rows(0)
    sx.set_store_sc1(-1)
    sx.set_sweep_mfma(-1)


if __name__ == "__main__":
    main()
