#!/bin/bash
# Round 3: matrix-core sweep at 64 slots with uniform buffer resources; padded rows; odd widths.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 ./tools/msweep_probe > gpurun_out/r03_msweep_probe3.txt 2>&1 && \
timeout -k 10 300 python3 -u tools/sweep_waves_ab.py 4096x11000 4096x12289 32768x10001 waves=1 rb=4 pol=1 mfma=0,1 \
    > gpurun_out/r03_mfma_sweep_ab4.log 2>&1
