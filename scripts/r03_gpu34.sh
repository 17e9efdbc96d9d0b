#!/bin/bash
# Round 3: two-stage multi-rank batches (fit check, two-pass activation): multi-rank parity,
# faults, then the probes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_multigpu_mode.py \
    tests/test_gpu_ipc.py tests/test_gpu_degenerate_faults.py -x -q --timeout 300 --timeout-method thread \
    -k "virtual or p2p or rank or multi or ipc or gpus or W or hang" > gpurun_out/r03_pytest_mr_v34.txt 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/p2p_probe.py config3 640 > gpurun_out/r03_multirank_config3_v34.txt 2>&1 && \
timeout -k 10 400 python3 -u tools/p2p_probe.py config5 320 > gpurun_out/r03_multirank_config5_v34.txt 2>&1
