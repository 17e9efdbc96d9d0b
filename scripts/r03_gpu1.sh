#!/bin/bash
# Round 3: the GPU suite on the new code (multi-GPU mode, split objective row, pruning), then the
# first probe (the reference's -t sweep, seed 110592, sweep grid sizes).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread \
    > gpurun_out/r03_pytest_gpu1.txt 2>&1
echo "pytest rc=$?" >> gpurun_out/r03_pytest_gpu1.txt
bash scripts/r03_probe1.sh
