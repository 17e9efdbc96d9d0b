"""The row-block sharded pivot protocol over torch.distributed (gloo, world_size 2, CPU).

The HIP engine shards the constraint rows into 512-aligned blocks and exchanges, per pivot,
(1) the 512-row ratio-tile winners (allgather, then the reference's pass-2 tree on every
rank) and (2) the pivot row (sum-allreduce where non-owners contribute -0.0, the exact
additive identity).  Here the same protocol runs on CPU ranks with the oracle's per-shard
functions, and must reproduce the single-process oracle bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle

TILE = 512


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _allgather(x):
    t = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64))
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return np.concatenate([o.numpy() for o in out])


def _phase(T, d, base, rank, world, rpr, row0, m, N):
    """solve() over shards (solver.cu:128-149 with the engine's exchange steps)."""
    rows = T.shape[0]
    slots = rpr // TILE
    big = np.finfo(np.float64).max
    pivots = 0
    while True:
        dmin_i, dmin = oracle.argmin(d[1:N])
        if not (dmin < 0 and abs(dmin) >= 1e-9):
            return oracle.FEASIBLE, pivots
        e = dmin_i
        colE = T[:, 1 + e].copy()
        tiles = np.zeros((slots, 3))
        tiles[:, 0] = big
        tiles[:, 1] = -1
        for k in range((rows + TILE - 1) // TILE):
            lo, hi = k * TILE, min(rows, (k + 1) * TILE)
            ratios = np.array([oracle.ratio(T[i, 0], colE[i]) for i in range(lo, hi)])
            v, idx = oracle.argmin_tile(ratios, row0 + lo)
            tiles[k] = (v, idx, float(np.any(colE[lo:hi] >= 1e-9)))
        allt = _allgather(tiles.reshape(-1)).reshape(-1, 3)  # world * slots tiles, global order
        if not allt[:, 2].any():
            return oracle.UNBOUNDED, pivots
        r, _ = oracle.argmin_pass2(allt[:, 0], allt[:, 1].astype(np.int64))
        own = row0 <= r < row0 + rows
        send = T[r - row0, :N].copy() if own else np.full(N, -0.0)
        t = torch.from_numpy(send)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        prow = t.numpy().copy()
        base[r] = e
        oracle.apply_update(T, d, prow, colE, (r - row0) if own else -1, prow[1 + e], dmin)
        pivots += 1


def _gemv(T, d, base, row0, rpr, world, m, N):
    rows = T.shape[0]
    coef = np.array([d[1 + base[row0 + i]] for i in range(rows)])
    slots = rpr // TILE
    part = np.zeros((slots, N))
    if rows:
        p = oracle.gemv_partials(np.ascontiguousarray(T[:, :N]), coef, N)
        part[:p.shape[0]] = p
    allp = _allgather(part.reshape(-1)).reshape(-1, N)
    oracle.gemv_apply(d[:N], allp[:(m + TILE - 1) // TILE])


def _worker(rank, world, port, n, m, seed, lo, hi, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    A, b, c = oracle.generate(n, m, seed, lo, hi)
    Tfull, d, base = oracle.build_phase1(A, b)
    rpr = ((m + world - 1) // world + TILE - 1) // TILE * TILE
    row0 = rank * rpr
    rows = max(0, min(rpr, m - row0))
    T = np.ascontiguousarray(Tfull[row0:row0 + rows])
    N1, N2 = 1 + n + 2 * m, 1 + n + m
    _gemv(T, d, base, row0, rpr, world, m, N1)
    st1, p1 = _phase(T, d, base, rank, world, rpr, row0, m, N1)
    status, p2, opt = None, 0, None
    if d[0] < 0 and abs(d[0]) >= 1e-9:
        status = oracle.INFEASIBLE
    elif any(n + m <= x < n + 2 * m for x in base):
        status = oracle.DEGENERATE
    else:
        d[1:1 + n] = -c
        d[1 + n:1 + n + m] = 0.0
        _gemv(T, d, base, row0, rpr, world, m, N2)
        status, p2 = _phase(T, d, base, rank, world, rpr, row0, m, N2)
        opt = d[0]
    rhs = np.zeros(rpr)
    rhs[:rows] = T[:, 0]
    allrhs = _allgather(rhs)[:m]
    x = np.zeros(n)
    for i in range(m):
        if base[i] < n:
            x[base[i]] = allrhs[i]
    if rank == 0:
        out.put((status, (p1, p2), opt, base.copy(), x))
    dist.destroy_process_group()


@pytest.mark.parametrize("n,m,seed,lo,hi", [(40, 600, 11, 1, 100), (30, 1100, 7, -100, 100), (256, 256, 25856, 1, 100)])
def test_two_rank_protocol_matches_single_process(n, m, seed, lo, hi):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, m, seed, lo, hi, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    status, pivots, opt, base, x = res
    A, b, c = oracle.generate(n, m, seed, lo, hi)
    ref = oracle.two_phase(A, b, c)
    assert status == ref["status"]
    assert pivots == ref["pivots"]
    assert np.array_equal(base, ref["base"])
    if status == oracle.FEASIBLE:
        assert np.float64(opt).view(np.uint64) == np.float64(ref["opt"]).view(np.uint64)
        assert np.array_equal(x.view(np.uint64), ref["x"].view(np.uint64))
