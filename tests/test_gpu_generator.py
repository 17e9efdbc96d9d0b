"""Device generator (jump-ahead XORWOW) vs the host generator and the oracle: bit-exact."""
import numpy as np
import pytest

import oracle
import simplexoncuda_amd as sx

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float64).view(np.uint64)


@pytest.mark.parametrize("n,m,seed,lo,hi", [(20, 10, 2010, 1, 100), (7, 5, 123456, -100, 100), (1, 1, 0, 0, 1),
                                            (2048, 1024, 205824, 1, 100), (300, 700, 99, -100, 100)])
def test_device_generator_matches_host(gpu, n, m, seed, lo, hi):
    A, b, c = sx.generateRandomProblemDevice(n, m, seed, lo, hi).arrays()
    Ah, bh, ch = sx.generateRandomProblem(n, m, seed, lo, hi).arrays()
    assert np.array_equal(bits(A), bits(Ah)) and np.array_equal(bits(b), bits(bh)) and np.array_equal(bits(c), bits(ch))


def test_device_generator_config5_far_jumps(gpu):
    """config 5 (n=8192, m=32768): the last rows sit 2^28 draws into the stream"""
    n, m, seed = 8192, 32768, 851968
    A, b, c = sx.generateRandomProblemDevice(n, m, seed, 1, 100).arrays()
    Ah, bh, ch = sx.generateRandomProblem(n, m, seed, 1, 100).arrays()
    assert np.array_equal(bits(b), bits(bh)) and np.array_equal(bits(c), bits(ch))
    assert np.array_equal(bits(A), bits(Ah))


@pytest.mark.parametrize("W", [1, 3])
def test_generated_tableau_matches_host_build(gpu, W):
    n, m, seed = 129, 1500, 77
    try:
        sx.set_virtual_ranks(W)
        T, d, base = sx.dev_build_phase1_generated(n, m, seed, -100, 100)
    finally:
        sx.set_virtual_ranks(1)
    A, bb, c = oracle.generate(n, m, seed, -100, 100)
    To, do, bo = oracle.build_phase1(A, bb)
    assert np.array_equal(bits(T), bits(To)) and np.array_equal(bits(d), bits(do)) and np.array_equal(base, bo)


def test_generated_session_matches_host_session(gpu):
    n, m, seed = 2048, 1024, 205824
    s1 = sx.Session(sx.generateRandomProblem(n, m, seed, 1, 100))
    s2 = sx.Session(generated=(n, m, seed, 1, 100))
    t1 = s1.pivots(100000)
    t2 = s2.pivots(100000)
    assert t1.pivots == t2.pivots == 2003
    assert bits(s1.objective()) == bits(s2.objective())
