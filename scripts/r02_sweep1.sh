#!/bin/bash
# Round-2 A/B of the one-column-per-thread sweep (k_sweep1) against k_sweep: its parity tests,
# the synthetic sweep bench and the in-loop chain A/B at configs 5 and 3.  Each GPU step has
# its own time limit; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== pytest ($(date +%T))"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider --timeout 300 \
    --timeout-method thread -k "one_column or large_batch_sweeps or two_region_layout" \
    > gpurun_out/pytest_sweep1.log 2>&1 || { tail -30 gpurun_out/pytest_sweep1.log; exit 1; }
tail -2 gpurun_out/pytest_sweep1.log
echo "== synthetic sweep A/B ($(date +%T))"
timeout -k 10 300 python -u tools/sweep_bench_ab.py 4096x8192 8192x8192 32768x9216 variants=1:4:0:2,1:4:0:1,1:2:0:1 \
    > gpurun_out/sweep1_ab.log 2>&1 || { tail -20 gpurun_out/sweep1_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/sweep1_ab.log
echo "== in-loop A/B ($(date +%T))"
timeout -k 10 400 python -u tools/chain_ab.py sweep=4:0:2,4:0:1,2:0:1 config=config5,config3 rounds=2 \
    > gpurun_out/sweep1_chain_ab.log 2>&1 || { tail -20 gpurun_out/sweep1_chain_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/sweep1_chain_ab.log
