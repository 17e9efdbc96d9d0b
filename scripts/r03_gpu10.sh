#!/bin/bash
# Round 3: readlane uniforms + last-leaving-slot shortcut in the history chains -- parity (whole
# parity file + faults), stage stamps, pivot-loop A/B of 32/64-pivot batches.
set -o pipefail
mkdir -p gpurun_out
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_degenerate_faults.py -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/r03_parity_v10.log 2>&1
rc=$?; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python3 -u tools/stage_stamps.py > gpurun_out/r03_stage_stamps2.txt 2>&1 && \
timeout -k 10 400 python3 -u tools/chain_ab.py batch=32,64 config=config5,config3 rounds=2 \
    > gpurun_out/r03_two_stage_chain_ab3.log 2>&1
