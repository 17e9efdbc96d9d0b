#!/bin/bash
# Round 3: the 64-slot matrix-core sweep with the next strip's tiles prefetched (one wave per
# SIMD, SIMPLEX_MSWEEP_PF=1) against the default; per-kernel sweep capacity cache fixed.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/sweep_kernels_ab.py 4096x8192 32768x9216 32768x10001 > gpurun_out/r03_pf0_sweeps.txt 2>&1 && \
SIMPLEX_MSWEEP_PF=1 timeout -k 10 200 python3 -u tools/sweep_kernels_ab.py 4096x8192 32768x9216 32768x10001 > gpurun_out/r03_pf1_sweeps.txt 2>&1 && \
SIMPLEX_MSWEEP_PF=1 timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread \
    -k "sweep or batch or large or two_phase" > gpurun_out/r03_pytest_pf1.txt 2>&1 && \
timeout -k 10 300 python3 -u bench.py > gpurun_out/r03_bench_pf0.log 2>&1 && \
SIMPLEX_MSWEEP_PF=1 timeout -k 10 300 python3 -u bench.py --no-update-bench > gpurun_out/r03_bench_pf1.log 2>&1
