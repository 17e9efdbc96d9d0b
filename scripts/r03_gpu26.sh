#!/bin/bash
# Round 3: the ratio side's one-round-trip objective answer (every objective tile's winner with
# its stored column + the pivot's details, the entering column's load issued before the history
# poll): parity (core files), stamps, bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_degenerate_faults.py \
    -x -q --timeout 150 --timeout-method thread > gpurun_out/r03_pytest_v26.txt 2>&1 && \
timeout -k 10 300 python3 -u tools/block_stamps.py config5,config3 > gpurun_out/r03_block_stamps_v26.txt 2>&1 && \
timeout -k 10 300 python3 -u tools/stage_stamps.py config5,config3 > gpurun_out/r03_stage_stamps_v26.txt 2>&1 && \
timeout -k 10 300 python3 -u bench.py > gpurun_out/r03_bench_v26.log 2>&1
