#!/bin/bash
# Round 3: one-stage batches (32 pivots) swept on the vector units vs the matrix cores, strip-major F.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u tools/chain_ab.py mfma=0,1 config=config3,config2,config4,config5 rounds=2 \
    > gpurun_out/r03_onestage_mfma_ab.txt 2>&1
