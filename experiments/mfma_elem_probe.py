"""The one element the matrix-core sweep got wrong (last row, last stored column of the 300 x 1100
instance): when does it change?  (diagnostic)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    import torch
    torch.cuda.set_device(0)
    import simplexoncuda_amd as sx
    import oracle
    A, b, c = oracle.generate(300, 1100, 11, 1, 100)
    T0, d0, base0 = oracle.build_phase1(A, b)
    oracle.update_objective(T0, d0, base0)
    print("initial", T0[1099, 1396:1401], T0[1098, 1400], T0.shape)
    for batch, fused in ((32, -1), (32, 0), (1, -1), (4, -1)):
        for k in (1, 2, 5, 32):
            for mf in (0, 1):
                Tg, dg, bg = T0.copy(), d0.copy(), base0.copy()
                sx.set_batch(batch)
                sx.set_fused(fused)
                sx.set_sweep_mfma(mf)
                st, done = sx.dev_pivots(Tg, dg, bg, k)
                sx.set_sweep_mfma(-1)
                sx.set_fused(-1)
                sx.set_batch(0)
                T, d, base = T0.copy(), d0.copy(), base0.copy()
                oracle.solve(T, d, base, max_pivots=k)
                bad = np.argwhere(Tg.view(np.uint64) != T.view(np.uint64))
                print(f"batch {batch} fused {fused} k {k} mfma {mf}: {len(bad)} differ; gpu row 1099 "
                      f"{Tg[1099, 1396:1401]} oracle {T[1099, 1396:1401]}", [tuple(x) for x in bad[:6]])


if __name__ == "__main__":
    main()
