"""The C-ABI library: loads without a GPU, exports every function include/*.h declares,
and its host-side code (generator, problem I/O) matches the oracle bit for bit."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle
import simplexoncuda_amd as sx
from conftest import GOLDEN, ROOT
from simplexoncuda_amd import _lib

HEADERS = ["macro.h", "problem.h", "tabular.h", "solver.h", "twoPhaseMethod.h", "simplex_hip.h"]


def declared_functions():
    names = set()
    for h in HEADERS:
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for line in src.splitlines():
            if line.startswith(("static", "typedef", "#", " ", "}")):
                continue
            mm = re.match(r"^[A-Za-z_][\w \*]*?[\s\*](\w+)\s*\(", line)
            if mm:
                names.add(mm.group(1))
    return names


def test_library_loads_and_exports_every_declared_symbol():
    lib = _lib.load()
    names = declared_functions()
    # the reference's drop-in surface must be there
    for must in ["twoPhaseMethod", "solve", "newTabular", "freeTabular", "printTableauToStream",
                 "readProblemFromFile", "readRandomProblemFromFile", "generateRandomProblem",
                 "printProblemToStream", "freeProblem", "enableBenchmarkMode", "disableBenchmarkMode"]:
        assert must in names
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert missing == []
    assert set(_lib.SIGNATURES) >= names


def test_problem_struct_layout():
    assert ctypes.sizeof(_lib.ProblemT) == 32
    assert _lib.ProblemT.vars.offset == 24 and _lib.ProblemT.constraints.offset == 28


@pytest.mark.parametrize("n,m,seed,lo,hi,rk", [
    (20, 10, 2010, 1, 100, 0), (8192 // 32, 4096 // 32, 823296, 1, 100, 0), (7, 5, 123456, -100, 100, 0),
    (13, 17, 4242, -100, 100, 1), (1, 1, 0, 0, 1, 0)])
def test_generator_matches_oracle(n, m, seed, lo, hi, rk):
    p = sx.generateRandomProblem(n, m, seed, lo, hi, rand_kind=rk)
    A, b, c = p.arrays()
    Ao, bo, co = oracle.generate(n, m, seed, lo, hi, rand_kind=rk)
    assert np.array_equal(A, Ao) and np.array_equal(b, bo) and np.array_equal(c, co)


def test_generated_values_in_range():
    p = sx.generateRandomProblem(64, 32, 99, 1, 100)
    A, b, c = p.arrays()
    for x in (A, b, c):
        assert x.min() >= 1.0 and x.max() <= 100.0


@pytest.mark.parametrize("name", ["smallProblem.txt", "infeasibleProblem.txt", "unboundedProblem.txt"])
def test_read_problem_file(name):
    path = os.path.join(GOLDEN, "examples", name)
    A, b, c = sx.readProblemFromFile(path).arrays()
    Ao, bo, co = oracle.read_problem_text(path)
    assert np.array_equal(A, Ao) and np.array_equal(b, bo) and np.array_equal(c, co)


def test_read_random_problem_file(tmp_path):
    f = tmp_path / "seed.txt"
    f.write_text("20 10 2010 1 100")
    A, b, c = sx.readRandomProblemFromFile(f).arrays()
    Ao, bo, co = oracle.generate(20, 10, 2010, 1, 100)
    assert np.array_equal(A, Ao) and np.array_equal(b, bo) and np.array_equal(c, co)


def test_print_problem(tmp_path):
    p = sx.readProblemFromFile(os.path.join(GOLDEN, "examples", "smallProblem.txt"))
    out = tmp_path / "p.txt"
    sx.printProblemToStream(p, out)
    txt = out.read_text()
    assert txt.startswith("max + 8.00 X1 + 10.00 X2 + 7.00 X3 \nsubject to \n")
    assert "+ 1.00 X1 + 3.00 X2 + 2.00 X3 <= 10.00" in txt


def _build_c_caller(tmp_path, compiler, std):
    import subprocess
    exe = tmp_path / f"drop_in_{compiler}"
    lib_dir = os.path.join(ROOT, "simplexoncuda_amd")
    cmd = [compiler, f"-std={std}", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "c", "drop_in_main.c"), "-L", lib_dir, "-lsimplex_hip",
           f"-Wl,-rpath,{lib_dir}", "-o", str(exe)]
    if compiler == "g++":
        cmd[1:1] = ["-x", "c++"]
    subprocess.run(cmd, check=True)
    return exe


@pytest.mark.parametrize("compiler,std", [("gcc", "c99"), ("g++", "c++17")])
def test_headers_compile_and_link_as_c_and_cxx(tmp_path, compiler, std):
    import subprocess
    exe = _build_c_caller(tmp_path, compiler, std)
    out = subprocess.run([str(exe), "host"], check=True, capture_output=True, text=True).stdout
    assert out.startswith("max + ") and "subject to" in out
    assert "compare(1e-10)=0 compare(-1)=-1" in out
