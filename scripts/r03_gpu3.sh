#!/bin/bash
# Round 3, third GPU run: the entering-column load issued first (fused batches), chain stamps,
# MFMA f64 probe with the corrected operand layout, uncached exchange-buffer bisect.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/r03_pytest_gpu3.txt 2>&1 && \
timeout -k 10 300 python3 -u tools/chain_ab.py rows=0 config=config5,config3 rounds=2 > gpurun_out/r03_chain3.txt 2>&1 && \
timeout -k 10 60 ./tools/mfma_f64_probe > gpurun_out/r03_mfma_probe2.txt 2>&1 && \
for mode in 3 1 2 0; do
    timeout -k 10 180 python3 -u tools/uncached_exchange_probe.py $mode >> gpurun_out/r03_uncached_bisect.txt 2>&1 || exit 1
done
