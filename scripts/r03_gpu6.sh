#!/bin/bash
# Round 3: the matrix-core sweep -- element probe, parity tests, sweep A/B, pivot-loop A/B.
set -o pipefail
mkdir -p gpurun_out
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 200 python3 -u tools/mfma_diff_probe.py > gpurun_out/r03_mfma_diff.txt 2>&1 || exit $?
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -v --timeout 120 --timeout-method thread \
    -k "matrix_core or two_region or batched_sweep" > gpurun_out/r03_mfma_tests3.log 2>&1
rc=$?; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python3 -u tools/sweep_waves_ab.py 4096x8192 32768x9216 1024x4096 waves=1,2 rb=4 pol=1 mfma=0,1 \
    > gpurun_out/r03_mfma_sweep_ab3.log 2>&1 && \
timeout -k 10 400 python3 -u tools/chain_ab.py mfma=0,1 config=config5,config3 rounds=2 \
    > gpurun_out/r03_mfma_chain_ab3.log 2>&1
