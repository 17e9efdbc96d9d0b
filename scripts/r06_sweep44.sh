#!/bin/bash
# Round 6: the 4x4x4 matrix-core sweep (msweep_steps44) -- parity subset, update kernel alone at two
# sizes, then a same-box A/B against the 16x16x4 steps (SIMPLEX_SWEEP44=0) on the driver's command.
source "$(dirname "$0")/gpu_step.sh"
step parity 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "${PK:-matrix_core or two_stage or layouts or subnormal or batched_sweep or sweep_grid or config5_pivots_match_oracle}" || exit $?
step ub 300 bash -c "for v in 1 0; do echo sweep44=\$v; SIMPLEX_SWEEP44=\$v python -u tools/update_bench_probe.py 4096 8192 32 64 || exit 1; SIMPLEX_SWEEP44=\$v python -u tools/update_bench_probe.py 16384 8192 32 64 || exit 1; done" || exit $?
cat $O/ub.log
TAG=${TAG}_ab REPS=${REPS:-2} VARIANTS="m44= m16=SIMPLEX_SWEEP44=0" bash scripts/r05_ab.sh
