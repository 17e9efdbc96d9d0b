#!/bin/bash
# Round 3: matrix-core sweep with one memory round trip per strip: sweep A/B, pivot loop A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/sweep_kernels_ab.py > gpurun_out/r03_sweep_kernels_ab.txt 2>&1 && \
timeout -k 10 400 python3 -u tools/chain_ab.py batch=32,64 config=config5,config3 rounds=2 \
    > gpurun_out/r03_two_stage_chain_ab5.log 2>&1
