"""Multi-process RCCL self-test of the sharded solver (run under torchrun).

Each rank drives its row block through libsimplex_hip.so; the per-pivot allgather and
allreduce go over the library's own RCCL communicator.  Rank 0 checks the answer against
the CPU oracle bit for bit.  On a 1-GPU box the ranks share device 0 (--same-device).
usage: torchrun --nproc-per-node W scripts/dist_selftest.py [--same-device] [--force-rccl]
(--force-rccl: run the exchange path over a real RCCL communicator even at W=1)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    same = "--same-device" in sys.argv
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = 0 if same else local
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    import simplexoncuda_amd as sx
    from simplexoncuda_amd import dist as sxdist

    sxdist.init_from_torch(dev, force_rccl="--force-rccl" in sys.argv)
    cases = [(300, 1100, 41100, 1, 100), (129, 1513, 77, -100, 100), (2048, 1024, 205824, 1, 100)]
    ok = True
    for mode, (n, m, seed, lo, hi) in [(md, c) for md in (1, 2) for c in cases]:
        sx.set_exchange_mode(mode)
        p = sx.generateRandomProblem(n, m, seed, lo, hi)
        t0 = time.time()
        got = sx.twoPhaseMethodEx(p)
        dt = time.time() - t0
        if rank == 0:
            import oracle

            A, b, c = p.arrays()
            ref = oracle.two_phase(A, b, c)
            good = (got.status == ref["status"] and tuple(got.pivots) == ref["pivots"]
                    and np.array_equal(got.base, ref["base"]))
            if got.status == sx.FEASIBLE:
                good = good and np.float64(got.optimal_value).view(np.uint64) == np.float64(ref["opt"]).view(np.uint64)
                good = good and np.array_equal(got.solution.view(np.uint64), ref["x"].view(np.uint64))
            ok = ok and good
            print(f"world={world} exchange_mode={mode} n={n} m={m}: status {got.status} pivots {got.pivots} "
                  f"{'BIT-EXACT' if good else 'MISMATCH'} vs oracle ({dt:.2f}s)", flush=True)
    sx.set_exchange_mode(0)
    # a timed session on the config-2 instance
    p = sx.generateRandomProblem(2048, 1024, 205824, 1, 100)
    s = sx.Session(p)
    s.pivots(20)
    dist.barrier()
    t = s.pivots(500, time_updates=8)
    if rank == 0:
        print(f"session: {t.pivots} pivots in {t.wall_ms:.2f} ms -> {t.pivots / t.wall_ms * 1e3:.0f} pivots/s, "
              f"rows/rank {t.local_rows}", flush=True)
    s.close()
    sxdist.finalize()
    dist.destroy_process_group()
    if rank == 0 and not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
