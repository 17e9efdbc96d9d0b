"""simplex_cli (the reference's main.cu front end) and the TIMER CSV (chrono.cu)."""
import csv
import json
import os
import subprocess

import pytest

from conftest import GOLDEN, ROOT

CLI = os.path.join(ROOT, "simplexoncuda_amd", "simplex_cli")


def run(args, tmp_path, **env):
    e = dict(os.environ, SIMPLEX_DATA_DIR=str(tmp_path), SIMPLEX_SOLUTION=str(tmp_path / "solution.txt"))
    e.update(env)
    return subprocess.run([CLI] + args, capture_output=True, text=True, env=e, timeout=600)


def test_cli_without_arguments(tmp_path):
    r = run([], tmp_path)
    assert r.returncode == 255 and "Not enough arguments!" in r.stderr


@pytest.mark.gpu
def test_cli_file(gpu, tmp_path):
    r = run(["-f", os.path.join(GOLDEN, "examples", "smallProblem.txt")], tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Problem solved!" in r.stdout
    assert (tmp_path / "solution.txt").read_text() == "8.000000\n0.000000\n0.000000\n\nOptimal value: 64.000000\n"
    r = run(["-f", os.path.join(GOLDEN, "examples", "infeasibleProblem.txt")], tmp_path)
    assert "Problem INFEASIBLE!" in r.stdout
    r = run(["-f", os.path.join(GOLDEN, "examples", "unboundedProblem.txt")], tmp_path)
    assert "Problem UNBOUNDED!" in r.stdout


@pytest.mark.gpu
def test_cli_random_seed_file_roundtrip(gpu, tmp_path):
    r = run(["-rs", "30", "20", "777"], tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    seeds = [f for f in os.listdir(tmp_path) if f.startswith("random_")]
    assert len(seeds) == 1
    assert (tmp_path / seeds[0]).read_text() == "30 20 777 -100 100"
    first = (tmp_path / "solution.txt").read_text() if "solved" in r.stdout else None
    r2 = run(["-rf", str(tmp_path / seeds[0])], tmp_path)
    assert r2.returncode == 0
    assert r2.stdout.splitlines()[-1] == r.stdout.splitlines()[-1]
    if first is not None:
        assert (tmp_path / "solution.txt").read_text() == first


@pytest.mark.gpu
def test_cli_benchmark_sweep_writes_reference_csv(gpu, tmp_path):
    """-t (capped at 512): benchmark_<n>_<m>.txt in the reference's format; the number of
    `solve` rows per phase equals the published pivot count + 1 (data/measures)."""
    r = run(["-t", "512"], tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    with open(os.path.join(GOLDEN, "published_pivots.json")) as f:
        pub = {(x["n"], x["m"]): x for x in json.load(f) if x["gpu"] == "rtx2070super"}
    for n in (256, 512):
        for m in (256, 512):
            path = tmp_path / f"benchmark_{n}_{m}.txt"
            rows = list(csv.reader(open(path)))
            assert rows[0] == ["vars", "contraints", "operation", "elapsed_time"]
            ops = [x[2] for x in rows[1:]]
            p1 = sum(1 for x in rows[1:] if x[2] == "solve" and int(x[0]) == 1 + n + 2 * m)
            p2 = sum(1 for x in rows[1:] if x[2] == "solve" and int(x[0]) == 1 + n + m)
            assert (p1 - 1, p2 - 1) == (pub[(n, m)]["p1_pivots"], pub[(n, m)]["p2_pivots"])
            expect = (["fillTableau", "gauss1"] + ["solve"] * p1 + ["checkDegeneracy", "costsVector", "gauss2"]
                      + ["solve"] * p2 + ["solution"])
            assert ops == expect
            assert all(int(x[1]) == m and float(x[3]) >= 0 for x in rows[1:])


@pytest.mark.gpu
def test_debug_trace(gpu, tmp_path):
    """SIMPLEX_DEBUG=1: the reference's DEBUG build output (tableau after fill, canonicalisation,
    every pivot and each phase), in its transposed print format"""
    r = run(["-f", os.path.join(GOLDEN, "examples", "smallProblem.txt")], tmp_path, SIMPLEX_DEBUG="1")
    assert r.returncode == 0, r.stdout + r.stderr
    out = r.stdout
    assert out.count("--------------- Tabular --------------") == 2 + 2 + 1 + 2 + 1  # fill, gauss, 2+2 pivots, 2 ends
    assert "Tableu nella situazione iniziale" in out and "Tableu dopo seconda esecuzione del solver" in out
    last = out[out.rindex("Tableu dopo seconda esecuzione del solver"):]
    assert "|\t 64.00000000000" in last and "Base\n3\t0\t" in last


def test_cli_rejects_bad_options(tmp_path):
    r = run(["--rand", "bsd", "-r", "3", "3", "1"], tmp_path)
    assert r.returncode == 255 and "--rand: expected msvc or glibc" in r.stderr
    r = run(["--frobnicate", "1", "-r", "3", "3", "1"], tmp_path)
    assert r.returncode == 255 and "Unknown option --frobnicate" in r.stderr
    r = run(["--gpus", "0", "-r", "3", "3", "1"], tmp_path)
    assert r.returncode == 255 and "--gpus: expected 1..8 GPUs, got 0" in r.stderr
    r = run(["--gpus", "9", "-r", "3", "3", "1"], tmp_path)  # (SIMPLEX_MAX_GPUS shards at most)
    assert r.returncode == 255 and "--gpus: expected 1..8 GPUs, got 9" in r.stderr


@pytest.mark.gpu
def test_cli_pivot_budget(gpu, tmp_path):
    """--pivot-budget K: twoPhaseMethodEx's per-phase cap (SIMPLEX_PIVOT_CAP), no solution written"""
    r = run(["--pivot-budget", "3", "-r", "300", "200", "5"], tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Pivot budget of 3 reached (phase pivots 3 + 0)" in r.stdout
    assert "Problem solved!" not in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["msvc", "glibc"])
def test_cli_rand_and_gpus(gpu, tmp_path, kind):
    """--rand picks the generator's rand(); --gpus 1 is the default device set. The CLI's
    objective equals the library's on the same generated instance"""
    import simplexoncuda_amd as sx
    r = run(["--gpus", "1", "--rand", kind, "-r", "60", "40", "99"], tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    p = sx.generateRandomProblem(60, 40, 99, -100, 100, rand_kind=sx.RAND_GLIBC if kind == "glibc" else sx.RAND_MSVC)
    try:
        st, _, opt = sx.twoPhaseMethod(p)
    finally:
        p.close()
    if st == sx.FEASIBLE:
        assert "Problem solved!" in r.stdout
        assert (tmp_path / "solution.txt").read_text().endswith("Optimal value: %f\n" % opt)
    else:
        assert "Problem solved!" not in r.stdout
