"""Diagnostic: dev_pivots on W = 2..4 virtual shards, then whole solves on W = 2 and 8,
against the oracle, with the exchange buffers in uncached memory by bit: argv[1] = 0 plain, 1 d, 2 U, 3 both
(simplex_set_uncached_exchange); argv[2] = "p2p" runs the peer-memory batch (default: the
per-pivot exchange of virtual shards).
usage: python tools/uncached_exchange_probe.py 0|1|2|3 [p2p]"""
import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import torch; torch.cuda.set_device(0)
import numpy as np, simplexoncuda_amd as sx, oracle
lib = sx.load(); print("lib", sx.LIB_PATH, flush=True)
unc = int(sys.argv[1]); lib.simplex_set_uncached_exchange(unc)
if len(sys.argv) > 2 and sys.argv[2] == "p2p": sx.set_p2p(1)
def phase1_state(n, m, seed, lo=1, hi=100):
    A, b, c = oracle.generate(n, m, seed, lo, hi)
    T, d, base = oracle.build_phase1(A, b)
    oracle.update_objective(T, d, base)
    return T, d, base
p = sx.generateRandomProblem(300, 1100, 300 * 100 + 1100, 1, 100)
A, b, c = p.arrays(); ref = oracle.two_phase(A, b, c)
for rep in range(3):
    for W in (2, 3, 4):
        T, d, base = phase1_state(200, 1500, 42)
        sx.set_virtual_ranks(W)
        Tg, dg, bg = T.copy(), d.copy(), base.copy()
        sx.dev_pivots(Tg, dg, bg, 60)
        sx.set_virtual_ranks(1)
    for W in (2, 8):
        sx.set_virtual_ranks(W)
        got = sx.twoPhaseMethodEx(p)
        sx.set_virtual_ranks(1)
        print(f"uncached={unc} p2p={lib.simplex_p2p_ready()} rep {rep} W={W}: {got.pivots} oracle {ref['pivots']} {'OK' if tuple(got.pivots)==ref['pivots'] else 'MISMATCH'}", flush=True)
