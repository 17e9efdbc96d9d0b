#!/bin/bash
# Diagnostic: what the leaving rows cost the matrix-core sweep (tools/_ab/libsimplex_dbg.so, a build
# of this tree whose launch reads SIMPLEX_SWEEP_DBG: bit 0 the strips store every row, bit 1 no
# fix-up, bit 2 no leaving-row bits loaded per strip).  Timing only: results are not checked.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/leave_dbg
mkdir -p $O
for d in ${DBGS:-0 1 2 3 4 7}; do
  echo "== dbg $d" | tee -a $O/out.txt
  for sz in "4096 8192" "16384 8192"; do
    SIMPLEX_LIB_PATH=tools/_ab/libsimplex_dbg.so SIMPLEX_SWEEP_DBG=$d timeout -k 10 120 python tools/update_bench_probe.py $sz 32 64 >> $O/out.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids $O/out.txt
