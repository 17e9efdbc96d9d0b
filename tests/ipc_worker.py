"""One rank of tests/test_gpu_ipc.py: a separate process that owns one row-block shard and runs
multi-rank fused batches whose hand-offs go through another process's memory (IPC handles),
the path simplex_dist_init's peer-memory mode uses across GPUs -- here without RCCL, so two
processes can share one GPU.  Line protocol on stdin/stdout with the parent:
  -> HANDLES <hex>      <- ALL <hex of every rank's handles, rank order>
  -> CONNECTED <rc>     <- GO
  -> DONE <status> <pivots>   <- SYNC
  -> SYNCED                   <- READ
  -> SAVED <hang recoveries> <fused batches>   (rows, d, base saved to <out>)   <- EXIT
usage: python tests/ipc_worker.py rank world n m seed lo hi pivots out.npz"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import oracle  # noqa: E402  (the input state; the parent checks the result)


def say(*a):
    print(*a, flush=True)


def main():
    rank, world, n, m, seed, lo, hi, pivots = (int(x) for x in sys.argv[1:9])
    out = sys.argv[9]
    import simplexoncuda_amd as sx
    lib = sx.load()
    lib.simplex_set_device(0)
    A, b, _ = oracle.generate(n, m, seed, lo, hi)
    T, d, base = oracle.build_phase1(A, b)
    oracle.update_objective(T, d, base)
    N1 = T.shape[1]
    rpr = ((m + world - 1) // world + 511) // 512 * 512
    r0, r1 = min(rank * rpr, m), min((rank + 1) * rpr, m)
    rows = np.ascontiguousarray(T[r0:r1]) if r1 > r0 else np.zeros((1, N1))
    hs = lib.simplex_ipc_handles_size()
    h = ctypes.create_string_buffer(hs)
    dp = ctypes.POINTER(ctypes.c_double)
    ip = ctypes.POINTER(ctypes.c_int)
    sess = lib.simplex_ipc_session_open(n, m, rank, world, rows.ctypes.data_as(dp), N1, d.ctypes.data_as(dp),
                                        base.ctypes.data_as(ip), h)
    if not sess:
        say("HANDLES FAIL")
        return 3
    say("HANDLES", h.raw.hex())
    line = sys.stdin.readline().split()
    assert line[0] == "ALL"
    rc = lib.simplex_ipc_session_connect(sess, bytes.fromhex(line[1]))
    say("CONNECTED", rc)
    assert sys.stdin.readline().strip() == "GO"
    t = sx.api._lib.TimingT()
    st = lib.simplex_session_pivots(sess, pivots, 0, ctypes.byref(t))
    say("DONE", st, t.pivots)
    # every rank's objective-row slice into every peer's row, between two barriers
    assert sys.stdin.readline().strip() == "SYNC"
    assert lib.simplex_session_sync_d(sess) == 0
    say("SYNCED")
    assert sys.stdin.readline().strip() == "READ"
    Tg = np.zeros((max(r1 - r0, 1), N1))
    dg = np.zeros(N1)
    bg = np.zeros(m, dtype=np.int32)
    nr = lib.simplex_session_rows(sess, Tg.ctypes.data_as(dp), N1, dg.ctypes.data_as(dp), bg.ctypes.data_as(ip))
    np.savez(out, T=Tg[:max(nr, 0)], d=dg, base=bg, r0=r0)
    say("SAVED", lib.simplex_hang_recoveries(), lib.simplex_fused_batches())
    assert sys.stdin.readline().strip() == "EXIT"
    lib.simplex_session_close(sess)
    return 0


if __name__ == "__main__":
    sys.exit(main())
