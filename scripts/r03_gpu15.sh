#!/bin/bash
# Round 3: same-box A/B of three builds of the matrix-core sweep in the config-5 pivot loop:
# A = committed (guards, per-pair loads), B = one round trip per strip, C = B without guards.
set -o pipefail
mkdir -p gpurun_out
for r in 0 1; do
for v in A B C; do
  if [ $v = C ]; then lib=simplexoncuda_amd/libsimplex_hip.so; else lib=tools/_ab/lib$v.so; fi
  echo "== variant $v round $r" >> gpurun_out/r03_sweep_variants_ab.txt
  SIMPLEX_LIB_PATH=$lib timeout -k 10 200 python3 -u tools/chain_ab.py batch=64 config=config5 rounds=1 \
      >> gpurun_out/r03_sweep_variants_ab.txt 2>&1 || exit $?
done
done
