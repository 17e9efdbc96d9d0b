"""Start-up cost of the multi-GPU self-check: wall time of the first
twoPhaseMethod call of a process on a small instance, with SIMPLEX_GPUS as given in the
environment (e.g. 0,0 or 0,0,0,0,0,0,0,0 -- virtual shards on one device) against a second call
in the same process.  usage: SIMPLEX_GPUS=0,0 python tools/selfcheck_time.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import simplexoncuda_amd as sx  # noqa: E402
from simplexoncuda_amd import _lib  # noqa: E402


def main():
    p = sx.generateRandomProblem(20, 10, 2010, 1, 100)
    t0 = time.perf_counter()
    sx.twoPhaseMethodEx(p)
    t1 = time.perf_counter()
    sx.twoPhaseMethodEx(p)
    t2 = time.perf_counter()
    print(f"SIMPLEX_GPUS={os.environ.get('SIMPLEX_GPUS', '')!r}: first call {t1 - t0:.3f} s, second {t2 - t1:.4f} s, "
          f"multi-GPU mode {_lib.load().simplex_multi_gpu_mode()}")


if __name__ == "__main__":
    main()
