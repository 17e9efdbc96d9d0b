"""Build the HIP product library (gfx950) and the CPU oracle, in-tree.

hipcc cross-compiles gfx950 code objects without a GPU, so this runs in the build
container and on the GPU box alike.  Outputs:
  simplexoncuda_amd/libsimplex_hip.so   the product (C-ABI of include/*.h)
  oracle/liboracle.so, oracle/oracle_cli the CPU checker (test infrastructure)
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "simplexoncuda_amd")
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libsimplex_hip.so")
SOURCES = ["sx_kernels.hip", "sx_generator.hip", "sx_engine.cpp", "sx_problem.cpp"]
HEADERS = ["sx_common.hpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SIMPLEX_OFFLOAD_ARCH", "gfx950")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_lib(force=False, verbose=False):
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps += [os.path.join(ROOT, "include", f) for f in os.listdir(os.path.join(ROOT, "include"))]
    if not force and not _stale(LIB, deps):
        return LIB
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-ffp-contract=off", "-Wall", "-I", os.path.join(ROOT, "include"), "-o", LIB]
    cmd += [os.path.join(CSRC, f) for f in SOURCES]
    cmd += ["-lrccl"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return LIB


CLI = os.path.join(PKG, "simplex_cli")


def build_cli(force=False):
    """simplex_cli: the reference's main.cu front end, linked against the library."""
    src = os.path.join(CSRC, "sx_cli.cpp")
    if not force and not _stale(CLI, [src, LIB]):
        return CLI
    cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-I", os.path.join(ROOT, "include"), src, "-L", PKG,
           "-lsimplex_hip", "-Wl,-rpath,$ORIGIN", "-o", CLI]
    subprocess.run(cmd, check=True)
    return CLI


def build_oracle(force=False):
    args = ["make", "-s", "-C", os.path.join(ROOT, "oracle")]
    if force:
        args.append("-B")
    subprocess.run(args, check=True)
    return os.path.join(ROOT, "oracle", "liboracle.so")


if __name__ == "__main__":
    build_lib(force="--force" in sys.argv, verbose=True)
    build_cli(force="--force" in sys.argv)
    build_oracle()
