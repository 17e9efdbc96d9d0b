#!/bin/bash
# Round 3: matrix-core sweep without the per-step guards: parity subset, sweep A/B, pivot loop A/B.
set -o pipefail
mkdir -p gpurun_out
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread \
    -k "two_stage or matrix_core or two_region or session" > gpurun_out/r03_parity_v14.log 2>&1
rc=$?; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python3 -u tools/sweep_kernels_ab.py > gpurun_out/r03_sweep_kernels_ab2.txt 2>&1 && \
timeout -k 10 400 python3 -u tools/chain_ab.py batch=32,64 config=config5,config3 rounds=2 \
    > gpurun_out/r03_two_stage_chain_ab6.log 2>&1
