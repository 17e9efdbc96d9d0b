#!/bin/bash
# Round 3: the 64-slot matrix-core sweep with lazily loaded fix-up operands: sweep A/B, then the
# whole GPU suite.
set -o pipefail
mkdir -p gpurun_out
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 200 python3 -u - > gpurun_out/r03_sweep64_ab.txt 2>&1 <<'PY' || exit $?
import torch
torch.cuda.set_device(0)
import simplexoncuda_amd as sx
for rnd in range(2):
    for rows, cols in ((4096, 8192), (32768, 9216), (32768, 10001), (4096, 11000)):
        for piv, mf in ((32, 0), (32, 1), (64, 1)):
            sx.set_sweep_mfma(mf)
            us, nb = sx.bench_sweep(rows, cols, 823296, 1, 100, piv, warmup=10, iters=40)
            print(f"round {rnd} {rows}x{cols} pivots={piv} mfma={mf}: {us:8.1f} us  frac {nb / us / 1e3 / 8000:.3f}"
                  f"  {us / piv:6.2f} us/pivot", flush=True)
sx.set_sweep_mfma(-1)
PY
timeout -k 10 1050 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
    > gpurun_out/r03_pytest_gpu_full_v12.log 2>&1
