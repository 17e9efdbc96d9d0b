"""The multi-rank fused batch (k_batch_mr) over a real 1-rank RCCL communicator, with its
buffers exchanged as IPC handles (own rank), checked bit for bit against the CPU oracle; then
the per-pivot RCCL exchange (both exchange modes) over the same communicator.  Run by
tests/test_gpu_parity.py in a child process (the library's distributed state is
process-global)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    import numpy as np

    import oracle
    import simplexoncuda_amd as sx
    from simplexoncuda_amd import _lib

    lib = _lib.load()
    uid = ctypes.create_string_buffer(lib.simplex_dist_unique_id_size())
    assert lib.simplex_dist_get_unique_id(uid) == 0
    sx.set_force_exchange(1)
    ok = True
    refs = {}  # (the oracle's whole solve once per instance: the three exchange modes share it)
    cases = [(300, 1100, 41100, 1, 100), (129, 1513, 77, -100, 100), (64, 128, 6528, 1, 100)]
    for label, p2p, mode in (("peer-memory fused batch", 1, 0), ("rccl tile allgather + row allreduce", 0, 1),
                             ("rccl row-gather", 0, 2)):
        sx.set_p2p(p2p)
        sx.set_exchange_mode(mode)
        assert lib.simplex_dist_init(0, 1, uid, 0) == 0
        for n, m, seed, lo, hi in cases:
            p = sx.generateRandomProblem(n, m, seed, lo, hi)
            got = sx.twoPhaseMethodEx(p)
            A, b, c = p.arrays()
            if (n, m, seed) not in refs:
                refs[(n, m, seed)] = oracle.two_phase(A, b, c)
            ref = refs[(n, m, seed)]
            good = (got.status == ref["status"] and tuple(got.pivots) == ref["pivots"]
                    and np.array_equal(got.base, ref["base"]))
            if got.status == sx.FEASIBLE:
                good = good and np.float64(got.optimal_value).view(np.uint64) == np.float64(ref["opt"]).view(np.uint64)
                good = good and np.array_equal(got.solution.view(np.uint64), ref["x"].view(np.uint64))
            ok = ok and good
            print(f"{label}: n={n} m={m} status {got.status} pivots {tuple(got.pivots)} "
                  f"{'bit-exact' if good else 'MISMATCH'}", flush=True)
        lib.simplex_dist_finalize()
        uid = ctypes.create_string_buffer(lib.simplex_dist_unique_id_size())
        assert lib.simplex_dist_get_unique_id(uid) == 0
    sx.set_p2p(-1)
    sx.set_exchange_mode(0)
    sx.set_force_exchange(0)
    print("ALL BIT-EXACT" if ok else "FAILED", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
