"""Diagnostic: the W = 8 divergence with the pending
pivot rows U in uncached memory, bisected on the current code.  Whole two-phase solves on W
virtual shards against the same solve on one shard, with U uncached (SIMPLEX_DIAG_UNCACHED_U=1)
or plain, per case: exchange form, slack compaction, layout, sweep kind, and an instance where
no shard is empty.
usage: python tools/uncached_u_bisect.py [case,...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

torch.cuda.set_device(0)
import simplexoncuda_amd as sx  # noqa: E402

lib = sx.load()

# (name, uncached U, knobs, (n, m)) -- 1100 rows on W = 8 leaves shards 3..7 empty (512-row
# blocks); 4000 rows gives every shard rows
CASES = {
    "ctl": (0, {"p2p": 0}, (300, 1100)),
    "unc": (1, {"p2p": 0}, (300, 1100)),
    "unc_nocompact": (1, {"p2p": 0, "compact": 0}, (300, 1100)),
    "unc_rowmajor": (1, {"p2p": 0, "blocked": 0}, (300, 1100)),
    "unc_vsweep": (1, {"p2p": 0, "sweep_mfma": 0}, (300, 1100)),
    "unc_p2p": (1, {"p2p": 1}, (300, 1100)),
    "fine": (0, {"p2p": 0, "fine": 1}, (300, 1100)),
    "fine_p2p": (0, {"p2p": 1, "fine": 1}, (300, 1100)),
    "unc_full": (1, {"p2p": 0}, (300, 4000)),
    "ctl_full": (0, {"p2p": 0}, (300, 4000)),
    # (run with SIMPLEX_DIAG_POISON=1: every allocation starts as NaN / -1 -- reads before writes)
    "poison_1": (0, {"p2p": 0}, (300, 1100)),
    "poison_1_p2p": (0, {"p2p": 1}, (300, 1100)),
    "poison_full": (0, {"p2p": 0}, (300, 4000)),
}


def knobs(k):
    # (tolerant of older trees without some of the setters: the bisect also runs earlier commits)
    for name, val in (("set_p2p", k.get("p2p", -1)), ("set_compact", k.get("compact", 1)),
                      ("set_blocked", k.get("blocked", -1)), ("set_sweep_mfma", k.get("sweep_mfma", -1)),
                      ("set_fine_pivot_rows", k.get("fine", -1))):
        if hasattr(sx, name):
            getattr(sx, name)(val)


def solve(n, m, W):
    p = sx.generateRandomProblem(n, m, n * 100 + m, 1, 100)
    sx.set_virtual_ranks(W)
    try:
        r = sx.twoPhaseMethodEx(p, 30000)  # (a cap: a diverged solve may cycle)
    finally:
        sx.set_virtual_ranks(1)
    return (r.status, tuple(r.pivots), float(r.optimal_value).hex(), r.base.tobytes())


def main():
    names = sys.argv[1].split(",") if len(sys.argv) > 1 else list(CASES)
    refs = {}
    for name in names:
        unc, k, (n, m) = CASES[name]
        os.environ["SIMPLEX_DIAG_UNCACHED_U"] = "0"
        knobs(k)
        if (n, m, str(k)) not in refs:
            refs[(n, m, str(k))] = solve(n, m, 1)
        ref = refs[(n, m, str(k))]
        os.environ["SIMPLEX_DIAG_UNCACHED_U"] = str(unc)
        for rep in range(int(os.environ.get("BISECT_REPS", "3"))):
            for W in (2, 8):
                got = solve(n, m, W)
                print(f"{name:14s} rep {rep} W={W}: {got[:2]} one shard {ref[:2]} "
                      f"{'OK' if got == ref else 'MISMATCH'}", flush=True)
        os.environ["SIMPLEX_DIAG_UNCACHED_U"] = "0"
        knobs({})


if __name__ == "__main__":
    main()
