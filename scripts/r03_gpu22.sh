#!/bin/bash
# Round 3: role-split batch loops + leaving-row words written without a load: parity (core
# files), the CLI options, per-block hand-off stamps (skew vs hop), stage stamps, the bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_degenerate_faults.py tests/test_cli.py \
    -x -q --timeout 150 --timeout-method thread --durations=15 > gpurun_out/r03_pytest_v22.txt 2>&1 && \
timeout -k 10 300 python3 -u tools/block_stamps.py config5,config3 > gpurun_out/r03_block_stamps.txt 2>&1 && \
timeout -k 10 300 python3 -u tools/stage_stamps.py config5,config3 > gpurun_out/r03_stage_stamps_v22.txt 2>&1 && \
timeout -k 10 300 python3 -u bench.py > gpurun_out/r03_bench_v22.log 2>&1
