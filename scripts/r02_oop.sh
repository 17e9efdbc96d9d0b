#!/bin/bash
# Round-2 probe: the register sweep in place vs out of place (read one buffer, write another)
# on synthetic matrices, after a quick parity pass of the in-place sweep.  Each GPU step has its
# own time limit; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== pytest ($(date +%T))"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider --timeout 300 \
    --timeout-method thread -k "batched_sweep or large_batch or session or two_region_layout" \
    > gpurun_out/pytest_oop.log 2>&1 || { tail -30 gpurun_out/pytest_oop.log; exit 1; }
tail -2 gpurun_out/pytest_oop.log
echo "== synthetic sweep in place vs out of place ($(date +%T))"
timeout -k 10 300 python -u tools/sweep_bench_ab.py 4096x8192 8192x8192 32768x9216 variants=1:4:0:2:0,1:4:0:2:1,0:4:0:2:1 \
    > gpurun_out/oop_ab.log 2>&1 || { tail -20 gpurun_out/oop_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/oop_ab.log
