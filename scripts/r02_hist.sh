#!/bin/bash
# Round-2 check of the branch-free history chains in the fused batch: the batch parity tests,
# then the chain A/B (hist_fast 1 vs 0, in-kernel stamps) and the driver's bench command.
# Each GPU step has its own time limit; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== pytest ($(date +%T))"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_degenerate_faults.py \
    tests/test_gpu_ipc.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_hist.log 2>&1 || { tail -30 gpurun_out/pytest_hist.log; exit 1; }
tail -3 gpurun_out/pytest_hist.log
echo "== chain A/B ($(date +%T))"
timeout -k 10 400 python -u tools/chain_ab.py hist_fast=1,0 config=config5,config3,config2 rounds=2 \
    > gpurun_out/chain_hist.log 2>&1 || { tail -20 gpurun_out/chain_hist.log; exit 1; }
cat gpurun_out/chain_hist.log
echo "== bench ($(date +%T))"
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_hist.log 2>&1 || { tail -20 gpurun_out/bench_hist.log; exit 1; }
tail -1 gpurun_out/bench_hist.log | cut -c1-600
