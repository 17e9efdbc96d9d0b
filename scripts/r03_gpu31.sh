#!/bin/bash
# Round 3: multi-rank batch -- records published granule-major over the ranks (value granules
# first), the W-fold U[q] stores issued behind the objective record: multi-rank parity, probes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_multigpu_mode.py \
    tests/test_gpu_ipc.py -x -q --timeout 200 --timeout-method thread -k "virtual or p2p or rank or multi or ipc or gpus or W" \
    > gpurun_out/r03_pytest_mr_v31.txt 2>&1 && \
timeout -k 10 400 python3 -u tools/p2p_probe.py config3 640 > gpurun_out/r03_multirank_config3_v31.txt 2>&1 && \
timeout -k 10 400 python3 -u tools/p2p_probe.py config5 320 > gpurun_out/r03_multirank_config5_v31.txt 2>&1
