#!/bin/bash
# Round 5: the 4x4x4 matrix-core sweep -- its arithmetic probe, parity subset, then a same-box A/B
# against the 16x16x4 sweep (SIMPLEX_SWEEP44=0).  Each GPU step under its own limit; a failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-s44}
mkdir -p $O
step() {
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -${TAILN:-4} "$O/$name.log" | cut -c1-300
    return $rc
}
[ "${SKIP_PROBE:-0}" = 1 ] || step probe 120 tools/_ab/mfma44_probe || exit $?
step parity 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "${PK:-matrix_core or two_stage or layouts or subnormal or batched_sweep or sweep_grid or config5_pivots_match_oracle}" || exit $?
step ub 300 bash -c "for v in 1 0; do for nl in 0 1; do echo sweep44=\$v noleave=\$nl; if [ \$nl = 1 ]; then export SIMPLEX_BENCH_NOLEAVE=1; else unset SIMPLEX_BENCH_NOLEAVE; fi; SIMPLEX_SWEEP44=\$v python -u tools/update_bench_probe.py 4096 8192 32 64 || exit 1; SIMPLEX_SWEEP44=\$v python -u tools/update_bench_probe.py 16384 8192 32 64 || exit 1; done; done" || exit $?
cat $O/ub.log
TAG=${TAG:-s44}_ab REPS=${REPS:-2} VARIANTS="m44= m16=SIMPLEX_SWEEP44=0" bash scripts/r05_ab.sh
