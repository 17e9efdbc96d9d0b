#!/bin/bash
# A GPU check of the current tree: core parity files, the sweep kernels on synthetic matrices,
# and the bench line (outputs under gpurun_out/, tag $1).
set -o pipefail
T=${1:-ab}
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_degenerate_faults.py \
    -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_pytest_$T.txt 2>&1 && \
timeout -k 10 200 python3 -u tools/sweep_kernels_ab.py 4096x8192 32768x9216 32768x10001 > gpurun_out/r03_sweeps_$T.txt 2>&1 && \
timeout -k 10 300 python3 -u bench.py --full-solves= > gpurun_out/r03_bench_$T.log 2>&1
