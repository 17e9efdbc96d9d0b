"""The one-process multi-GPU mode of the drop-in ("Multi-GPU is internal: the
caller still sees one synchronous call.  Device list comes from the env/flag SIMPLEX_GPUS"), and
bench.py's --gpus N (needs an MI355X).

On a one-GPU box the device list maps every shard onto GPU 0 ("0,0,0"): the same shards,
exchanges and self-check as on N GPUs, minus the cross-device memory.  A list naming a GPU that
is not visible must fail loudly, and `bench.py --gpus N` must refuse to print a line for fewer
GPUs than asked.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
from conftest import ROOT, two_phase_ref

pytestmark = pytest.mark.gpu

CHILD = r"""
import sys, json
sys.path.insert(0, {root!r})
import numpy as np
import simplexoncuda_amd as sx
lib = sx.load()
sx.set_replicated_objective({repl})
p = sx.generateRandomProblem({n}, {m}, {seed}, {lo}, {hi})
r = sx.twoPhaseMethodEx(p)
print(json.dumps({{"gpus": sx.gpus(), "status": r.status, "pivots": list(r.pivots), "opt": float(r.optimal_value).hex(),
                  "x": [float(v).hex() for v in r.solution], "base": [int(b) for b in r.base],
                  "p2p_ready": lib.simplex_p2p_ready(), "fused": lib.simplex_fused_batches(),
                  "hangs": lib.simplex_hang_recoveries()}}))
"""


def run_child(env_gpus, n, m, seed, lo, hi, repl=-1):
    env = dict(os.environ, SIMPLEX_GPUS=env_gpus)
    code = CHILD.format(root=ROOT, n=n, m=m, seed=seed, lo=lo, hi=hi, repl=repl)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=240)


@pytest.mark.parametrize("gpus,repl", [("0,0", -1), ("0,0,0", -1), ("0,0,0,0,0,0,0,0", -1), ("0,0", 1), ("0,0,0,0", 1)])
@pytest.mark.parametrize("n,m,seed,lo,hi", [(300, 1100, 41100, 1, 100), (129, 1513, 77, -100, 100)])
def test_unchanged_caller_gets_shards_from_env(gpu, gpus, repl, n, m, seed, lo, hi):
    """(repl 1: the replicated objective -- the default across GPUs -- forced on the one device,
    self-check included)"""
    import json
    r = run_child(gpus, n, m, seed, lo, hi, repl)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    got = json.loads(r.stdout.strip().splitlines()[-1])
    assert got["gpus"] == [int(x) for x in gpus.split(",")]
    A, b, c = oracle.generate(n, m, seed, lo, hi)
    ref = two_phase_ref(A, b, c)
    assert got["status"] == ref["status"] and tuple(got["pivots"]) == ref["pivots"]
    assert np.array_equal(np.array(got["base"]), ref["base"])
    if ref["status"] == 0:
        assert got["opt"] == float(ref["opt"]).hex()
        assert got["x"] == [float(v).hex() for v in ref["x"]]
    # the mode's start-up self-check passed: the batches ran on the peer-memory path, none re-run
    assert got["p2p_ready"] == 1 and got["fused"] > 0 and got["hangs"] == 0


CHILD_P2P_OFF_ON = r"""
import sys, json
sys.path.insert(0, {root!r})
import simplexoncuda_amd as sx
lib = sx.load()
out = {{}}
for mode in (0, -1):
    sx.set_p2p(mode)
    f0 = lib.simplex_fused_batches()
    r = sx.twoPhaseMethodEx(sx.generateRandomProblem(300, 1100, 41100, 1, 100))
    out[str(mode)] = {{"status": r.status, "pivots": list(r.pivots), "mode": lib.simplex_multi_gpu_mode(),
                      "p2p_ready": lib.simplex_p2p_ready(), "fused": lib.simplex_fused_batches() - f0}}
print(json.dumps(out))
"""


def test_self_check_with_peer_memory_off_then_on(gpu):
    """simplex_set_p2p(0) checks only the per-pivot exchange: that result (1) must not be reused once
    peer memory is enabled again -- the next solve runs the full check and the peer-memory batches
    """
    import json
    env = dict(os.environ, SIMPLEX_GPUS="0,0")
    r = subprocess.run([sys.executable, "-c", CHILD_P2P_OFF_ON.format(root=ROOT)], capture_output=True, text=True,
                       env=env, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "disagree" not in r.stderr
    got = json.loads(r.stdout.strip().splitlines()[-1])
    A, b, c = oracle.generate(300, 1100, 41100, 1, 100)
    ref = two_phase_ref(A, b, c)
    for mode in ("0", "-1"):
        assert got[mode]["status"] == ref["status"] and tuple(got[mode]["pivots"]) == ref["pivots"]
    assert got["0"]["mode"] == 1 and got["0"]["p2p_ready"] == 0
    assert got["-1"]["mode"] == 2 and got["-1"]["p2p_ready"] == 1 and got["-1"]["fused"] > 0


def test_missing_device_is_fatal(gpu):
    import torch
    n_vis = torch.cuda.device_count()
    r = run_child(",".join(str(i) for i in range(n_vis + 1)), 20, 10, 2010, 1, 100)
    assert r.returncode != 0
    assert f"SIMPLEX_GPUS: device {n_vis} requested but {n_vis} visible" in r.stdout + r.stderr


def test_bench_refuses_more_gpus_than_visible(gpu):
    import torch
    n_vis = torch.cuda.device_count()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "SIMPLEX_GPUS")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n_vis + 1), "--steps", "1",
                        "--warmup", "0"], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 2, r.stdout[-2000:] + r.stderr[-2000:]
    assert f"--gpus {n_vis + 1} needs {n_vis + 1} GPUs, {n_vis} visible" in r.stderr
    assert r.stdout.strip() == ""  # no bench line
