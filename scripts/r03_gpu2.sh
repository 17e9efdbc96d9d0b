#!/bin/bash
# Round 3, second GPU run: the suite on the split-hand-off fused batches, chain stamps, the bench
# line, the MFMA f64 exactness probe, the uncached-reuse probe and a wider sweep-grid A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r03_pytest_gpu2.txt 2>&1 && \
timeout -k 10 300 python3 -u tools/chain_ab.py rows=0 config=config5,config3 rounds=2 > gpurun_out/r03_chain2.txt 2>&1 && \
timeout -k 10 400 python3 -u bench.py > gpurun_out/r03_bench2.json 2> gpurun_out/r03_bench2.err && \
timeout -k 10 60 ./tools/mfma_f64_probe > gpurun_out/r03_mfma_probe.txt 2>&1 && \
timeout -k 10 120 ./tools/uncached_reuse_probe > gpurun_out/r03_uncached_reuse.txt 2>&1 && \
timeout -k 10 120 ./tools/uncached_reuse_probe --writeback >> gpurun_out/r03_uncached_reuse.txt 2>&1 && \
timeout -k 10 400 python3 -u tools/sweep_waves_ab.py 4096x8192 8192x8192 32768x9216 waves=1,1.25,1.5,2 rb=2,4 \
    > gpurun_out/r03_sweep_waves2.log 2>&1
