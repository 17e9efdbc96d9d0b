#!/bin/bash
# Round 3: strip-major F layout -- parity (every F reader/writer), then same-box A/B against the
# previous build (tools/_ab/libB.so) in the sweep bench and the pivot loop.
set -o pipefail
mkdir -p gpurun_out
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread \
    -k "two_stage or matrix_core or two_region or batched_sweep or large_batch or p2p or exchange or pivots" \
    > gpurun_out/r03_parity_v16.log 2>&1
rc=$?; if fatal $rc; then exit $rc; fi
for r in 0 1; do for v in B C; do
  if [ $v = C ]; then lib=simplexoncuda_amd/libsimplex_hip.so; else lib=tools/_ab/lib$v.so; fi
  echo "== variant $v round $r" >> gpurun_out/r03_flayout_ab.txt
  SIMPLEX_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/chain_ab.py batch=32,64 config=config5,config3 rounds=1 \
      >> gpurun_out/r03_flayout_ab.txt 2>&1 || exit $?
done; done
timeout -k 10 300 python3 -u tools/sweep_kernels_ab.py 4096x8192 32768x9216 > gpurun_out/r03_sweep_kernels_ab3.txt 2>&1
