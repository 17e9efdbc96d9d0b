"""Where does the matrix-core sweep differ from the oracle on virtual shards?  (diagnostic)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    import torch
    torch.cuda.set_device(0)
    import simplexoncuda_amd as sx
    import oracle  # noqa
    A, b, c = oracle.generate(300, 1100, 11, 1, 100)
    for W, p2p, mfma, k in ((1, -1, 1, 150), (2, 1, 0, 150), (2, 1, 1, 150), (2, 0, 1, 150), (2, 1, 1, 32),
                            (2, 1, 1, 64)):
        T, d, base = oracle.build_phase1(A, b)
        oracle.update_objective(T, d, base)
        Tg, dg, bg = T.copy(), d.copy(), base.copy()
        sx.set_batch(32)
        sx.set_virtual_ranks(W)
        sx.set_p2p(p2p)
        sx.set_sweep_mfma(mfma)
        st, done = sx.dev_pivots(Tg, dg, bg, k)
        sx.set_virtual_ranks(1)
        sx.set_p2p(-1)
        sx.set_sweep_mfma(-1)
        oracle.solve(T, d, base, max_pivots=k)
        bad = np.argwhere(Tg.view(np.uint64) != T.view(np.uint64))
        print(f"W={W} p2p={p2p} mfma={mfma} k={k}: done {done}, {len(bad)} T entries differ, d same "
              f"{np.array_equal(dg.view(np.uint64), d.view(np.uint64))}, base same {np.array_equal(bg, base)}")
        for i, j in bad[:12]:
            print(f"   ({i},{j}) gpu {Tg[i, j]!r} oracle {T[i, j]!r}")
        if len(bad):
            print("   rows", np.unique(bad[:, 0])[:40], "cols", np.unique(bad[:, 1])[:40])


if __name__ == "__main__":
    main()
