"""The multi-rank fused batch across PROCESSES on real memory: W ranks, each a separate process
(tests/ipc_worker.py) owning one row-block shard on the same GPU, whose k_batch_mr launches
hand off through each other's buffers mapped by IPC handles (hipIpcGetMemHandle /
hipIpcOpenMemHandle) -- the mechanism the RCCL ranks use across GPUs, minus RCCL (which
refuses two ranks on one device).  The assembled tableau, objective row and basis after K
phase-1 pivots must equal the CPU oracle's bit for bit (solver.cu:78-126).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
from conftest import ROOT

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


def run_ranks(tmp_path, world, n, m, seed, lo, hi, pivots):
    worker = os.path.join(ROOT, "tests", "ipc_worker.py")
    procs, outs = [], []
    env = dict(os.environ)
    for r in range(world):
        out = str(tmp_path / f"rank{r}.npz")
        outs.append(out)
        procs.append(subprocess.Popen([sys.executable, "-u", worker, str(r), str(world), str(n), str(m), str(seed),
                                       str(lo), str(hi), str(pivots), out], stdin=subprocess.PIPE,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env))
    try:
        def expect(p, tag):
            line = p.stdout.readline().split()
            assert line and line[0] == tag, (tag, line, p.stderr.read() if p.poll() is not None else "")
            return line[1:]

        handles = [expect(p, "HANDLES")[0] for p in procs]
        assert "FAIL" not in handles
        for p in procs:
            p.stdin.write("ALL " + "".join(handles) + "\n")
            p.stdin.flush()
        rcs = [int(expect(p, "CONNECTED")[0]) for p in procs]
        assert rcs == [0] * world, rcs  # every rank mapped its peers and the fused grid fits
        for p in procs:
            p.stdin.write("GO\n")
            p.stdin.flush()
        done = [expect(p, "DONE") for p in procs]
        for step, reply in (("SYNC", "SYNCED"), ("READ", "SAVED")):
            for p in procs:
                p.stdin.write(step + "\n")
                p.stdin.flush()
            got = [expect(p, reply) for p in procs]
        # every rank stayed on the peer-memory path: fused batches ran, none timed out and was re-run
        for hr, fb in got:
            assert int(hr) == 0 and int(fb) > 0, (hr, fb)
        for p in procs:
            p.stdin.write("EXIT\n")
            p.stdin.flush()
        for p in procs:
            assert p.wait(timeout=120) == 0, p.stderr.read()
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return [(int(s), int(k)) for s, k in done], [np.load(o) for o in outs]


@pytest.mark.parametrize("world,n,m,seed,lo,hi,pivots", [
    (2, 300, 1100, 41100, 1, 100, 150),      # 1024 + 76 rows: ratio tiles on both ranks
    (2, 2048, 1024, 205824, 1, 100, 200),    # config 2's instance: 512 + 512 rows
    (2, 129, 1513, 77, -100, 100, 120),      # negated rows (b < 0 quirk)
    (3, 300, 1100, 41100, 1, 100, 100),      # 512 + 512 + 76 rows
    (2, 64, 128, 6528, 1, 100, 10000),       # the whole phase 1, ending mid-batch
])
def test_multiprocess_peer_memory_batches(gpu, tmp_path, world, n, m, seed, lo, hi, pivots):
    A, b, _ = oracle.generate(n, m, seed, lo, hi)
    T, d, base = oracle.build_phase1(A, b)
    oracle.update_objective(T, d, base)
    st_o, k_o = oracle.solve(T, d, base, max_pivots=pivots)
    done, res = run_ranks(tmp_path, world, n, m, seed, lo, hi, pivots)
    for st, k in done:
        assert k == k_o
        assert (st == -10) == (st_o == oracle.PIVOT_CAP) and (st == st_o or st_o == oracle.PIVOT_CAP)
    Tg = np.concatenate([r["T"] for r in res if r["T"].shape[0] > 0])
    assert Tg.shape == T.shape
    assert np.array_equal(bits(Tg), bits(T))
    for r in res:  # every rank holds the whole objective row and basis
        assert np.array_equal(bits(r["d"]), bits(d))
        assert np.array_equal(r["base"], base)
