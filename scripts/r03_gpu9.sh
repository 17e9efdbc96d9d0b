#!/bin/bash
# Round 3: plain F / U stores in the fused batch (L2 write-back at the stage switch and at exit):
# parity, then the pivot-loop A/B of 32- and 64-pivot batches.
set -o pipefail
mkdir -p gpurun_out
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread \
    -k "two_stage or batched_sweep or compaction or fused or pivots_bit_exact" \
    > gpurun_out/r03_two_stage_tests2.log 2>&1
rc=$?; if fatal $rc; then exit $rc; fi
timeout -k 10 400 python3 -u tools/chain_ab.py batch=32,64 config=config5,config3 rounds=2 \
    > gpurun_out/r03_two_stage_chain_ab2.log 2>&1
