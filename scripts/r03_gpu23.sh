#!/bin/bash
# Round 3: the entering column's stored position in the objective record, its load issued
# after the pivot's stores: parity (core files), per-block stamps, stage stamps, the bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_degenerate_faults.py \
    -x -q --timeout 150 --timeout-method thread > gpurun_out/r03_pytest_v23.txt 2>&1 && \
timeout -k 10 300 python3 -u tools/block_stamps.py config5,config3 > gpurun_out/r03_block_stamps_v23.txt 2>&1 && \
timeout -k 10 300 python3 -u tools/stage_stamps.py config5,config3 > gpurun_out/r03_stage_stamps_v23.txt 2>&1 && \
timeout -k 10 300 python3 -u bench.py > gpurun_out/r03_bench_v23.log 2>&1
