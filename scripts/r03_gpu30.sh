#!/bin/bash
# Round 3: aborts inside a running fused batch (hang-inject slot hook): fault tests, then the bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_degenerate_faults.py -v --timeout 150 --timeout-method thread \
    > gpurun_out/r03_pytest_faults_v30.txt 2>&1 && \
timeout -k 10 300 python3 -u bench.py > gpurun_out/r03_bench_v30.log 2>&1
