#!/bin/bash
# Round 6: whole twoPhaseMethod solves of configs 4 and 5 with the 4x4x4 vs 16x16x4 matrix steps
source "$(dirname "$0")/gpu_step.sh"
for rep in 1 2; do
  for v in 1 0; do
    step fs_m44_${v}_$rep 200 env SIMPLEX_SWEEP44=$v python -u tools/full_solve.py config4 config5 || exit $?
  done
done
grep -h "" $O/fs_*.log | grep -v amdgpu.ids
