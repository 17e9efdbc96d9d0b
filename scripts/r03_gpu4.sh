#!/bin/bash
# Round 3: MFMA sweep prototype (K = 32 / 64, bit-exactness vs the VALU chain, bandwidth) and the
# VALU sweep's cache-policy A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 ./tools/msweep_probe > gpurun_out/r03_msweep_probe.txt 2>&1 && \
timeout -k 10 400 python3 -u tools/sweep_waves_ab.py 4096x8192 32768x9216 waves=1 rb=4 pol=1,0,2,3,4 \
    > gpurun_out/r03_sweep_policy.log 2>&1
