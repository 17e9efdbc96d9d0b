"""Grid size of the 32-slot update kernel (k_msweep<8>) on the synthetic update bench: blocks as a
multiple of the resident capacity (simplex_set_update_waves; 1.0 = the engine's rule, 2/3 of it for
the one-stage kernel).  (experiment helper)"""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))))
import torch  # noqa: E402

torch.cuda.set_device(0)
import simplexoncuda_amd as sx  # noqa: E402

for rows in (16384, 4096):
    for w in (1.0, 0.5, 0.999, 1.333, 2.0, 3.0):
        sx.set_update_waves(w)
        runs = [sx.bench_sweep(rows, 8192, 823296, 1, 100, 32, warmup=10, iters=50) for _ in range(3)]
        us, nbytes = sorted(runs)[1]
        print(f"{rows}x8192 k=32 waves {w}: {us:.1f} us, {nbytes / us / 1e3 / 8000:.3f} of 8 TB/s", flush=True)
sx.set_update_waves(1.0)
