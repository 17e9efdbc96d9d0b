import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")

_TWO_PHASE = {}


def two_phase_ref(A, b, c):
    """oracle.two_phase, computed once per instance in a session (several GPU tests check
    different engine modes against the same whole solve); arrays returned as copies."""
    import hashlib

    import numpy as np
    import oracle

    arrs = [np.ascontiguousarray(x, dtype=np.float64) for x in (A, b, c)]
    key = hashlib.sha1(b"".join(x.tobytes() for x in arrs) + repr(arrs[0].shape).encode()).hexdigest()
    if key not in _TWO_PHASE:
        _TWO_PHASE[key] = oracle.two_phase(*arrs)
    return {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in _TWO_PHASE[key].items()}


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP library)")
    config.addinivalue_line("markers", "slow: long CPU oracle runs")


@pytest.fixture(scope="session", autouse=True)
def _built():
    from simplexoncuda_amd.build import build_cli, build_lib, build_oracle

    build_oracle()
    build_lib()
    build_cli()


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    return 0
