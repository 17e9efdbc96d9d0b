#!/bin/bash
# Round 3, second GPU run: the suite on the split-hand-off fused batch, chain stamps, the bench
# line, the MFMA f64 exactness probe and a wider sweep-grid A/B; last, `--gpus 2` on a 1-GPU box
# (must exit non-zero with a clear message).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r03_pytest_gpu2.txt 2>&1 && \
timeout -k 10 300 python3 -u tools/chain_ab.py rows=0 config=config5,config3 rounds=2 > gpurun_out/r03_chain2.txt 2>&1 && \
timeout -k 10 400 python3 -u bench.py > gpurun_out/r03_bench2.json 2> gpurun_out/r03_bench2.err && \
timeout -k 10 60 ./tools/mfma_f64_probe > gpurun_out/r03_mfma_probe.txt 2>&1 && \
timeout -k 10 400 python3 -u tools/sweep_waves_ab.py 4096x8192 8192x8192 32768x9216 waves=1,1.25,1.5,2 rb=2,4 \
    > gpurun_out/r03_sweep_waves2.log 2>&1 && \
{ timeout -k 10 120 python3 -u bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/r03_bench_gpus2.out 2>&1; \
  echo "rc=$?" >> gpurun_out/r03_bench_gpus2.out; }
