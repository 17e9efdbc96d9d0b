"""Pivot rate of the multi-rank paths on ONE GPU (diagnostic): virtual shards with the per-pivot
exchange vs the peer-memory fused batch, and the fused multi-rank kernel at W = 1 (force).

Virtual shards share the one GPU (every shard's sweep runs on it), so the W > 1 rates show the
hand-off costs, not a multi-GPU speed-up.
usage: python tools/p2p_probe.py [config] [pivots] [--repl]
  --repl: the peer-memory lines with the split objective (each rank its share of the objective
  tiles) and with the replicated one (every rank all of them, simplex_set_replicated_objective)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def run(sx, n, m, seed, k, W, p2p, force=0, batch=0, repl=-1):
    sx.set_replicated_objective(repl)
    sx.set_virtual_ranks(W)
    sx.set_p2p(p2p)
    sx.set_force_exchange(force)
    sx.set_batch(batch)
    try:
        s = sx.Session(generated=(n, m, seed, 1, 100))
        s.pivots(64)
        t = s.pivots(k, time_updates=1)
        s.close()
    finally:
        sx.set_virtual_ranks(1)
        sx.set_p2p(-1)
        sx.set_force_exchange(0)
        sx.set_batch(0)
        sx.set_replicated_objective(-1)
    return t


def main():
    import torch
    torch.cuda.set_device(0)
    import simplexoncuda_amd as sx
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    cfg = args[0] if args else "config3"
    k = int(args[1]) if len(args) > 1 else 640
    n, m, seed = bench.CONFIGS[cfg]
    if "--repl" in sys.argv:
        cases = [(1, -1, 0, 0, -1)] + [(W, 1, 0, 0, r) for W in (2, 3, 4, 8) for r in (0, 1)]
    else:
        cases = [(W, p2p, force, batch, -1) for W, p2p, force, batch in
                 [(1, -1, 0, 0), (1, -1, 0, 32), (1, 1, 1, 32), (2, 0, 0, 0), (2, 1, 0, 0), (3, 1, 0, 0), (4, 1, 0, 0),
                  (8, 1, 0, 0)]]
    for W, p2p, force, batch, repl in cases:
        f0 = sx.load().simplex_fused_batches()
        t = run(sx, n, m, seed, k, W, p2p, force, batch, repl)
        fused = sx.load().simplex_fused_batches() - f0
        per = t.wall_ms * 1e3 / max(t.pivots, 1)
        sw = t.update_ms * 1e3 / max(t.pivots, 1)  # (shard 0's sweeps)
        print(f"{cfg} W={W} p2p={p2p} force_exchange={force} batch={batch or 'default'} repl={repl} fused={fused}: "
              f"{t.pivots / t.wall_ms * 1e3:9.1f} pivots/s ({per:7.2f} us/pivot = shard-0 sweep {sw:6.2f} + rest "
              f"{per - sw:6.2f}; sweep {t.update_ms * 1e3 / max(t.update_launches, 1):8.1f} us) status {t.status}",
              flush=True)


if __name__ == "__main__":
    main()
