#!/bin/bash
# Round 3: the one-shard batch's U[q] store behind the objective record: parity (core files),
# stage stamps, bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_degenerate_faults.py tests/test_gpu_large.py \
    -x -q --timeout 150 --timeout-method thread > gpurun_out/r03_pytest_v32.txt 2>&1 && \
timeout -k 10 300 python3 -u tools/stage_stamps.py config5,config3 > gpurun_out/r03_stage_stamps_v32.txt 2>&1 && \
timeout -k 10 300 python3 -u bench.py > gpurun_out/r03_bench_v32.log 2>&1
