#!/bin/bash
# Round 3: the whole GPU suite on the final sweep / batch defaults.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1150 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
    > gpurun_out/r03_pytest_gpu_full_v18.log 2>&1
