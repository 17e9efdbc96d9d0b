#!/bin/bash
# Round 3: the whole GPU suite on the final defaults, with per-test durations.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1150 python3 -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread --durations=60 \
    > gpurun_out/r03_pytest_gpu_full_v21.log 2>&1
