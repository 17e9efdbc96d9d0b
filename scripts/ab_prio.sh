#!/bin/bash
# Round 3: the 64-slot sweep's matrix steps at wave priority 1 (SIMPLEX_MSWEEP_PRIO=1) vs default.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/sweep_kernels_ab.py 4096x8192 32768x9216 32768x10001 > gpurun_out/r03_prio0_sweeps.txt 2>&1 && \
SIMPLEX_MSWEEP_PRIO=1 timeout -k 10 200 python3 -u tools/sweep_kernels_ab.py 4096x8192 32768x9216 32768x10001 > gpurun_out/r03_prio1_sweeps.txt 2>&1 && \
timeout -k 10 300 python3 -u bench.py --no-update-bench --full-solves= --no-cpu-baseline > gpurun_out/r03_bench_prio0.log 2>&1 && \
SIMPLEX_MSWEEP_PRIO=1 timeout -k 10 300 python3 -u bench.py --no-update-bench --full-solves= --no-cpu-baseline > gpurun_out/r03_bench_prio1.log 2>&1
