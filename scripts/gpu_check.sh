#!/bin/bash
# GPU-box round: parity tests, smoke, bench.  Each GPU step has its own time limit; a crash,
# abort or timeout ends the script (a plain test failure, exit 1, does not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -5 "gpurun_out/$name.log"
    return $rc
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --maxfail=5 -p no:cacheprovider --timeout 300 --timeout-method thread
rc=$?; [ $rc -gt 1 ] && exit $rc
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 600 python bench.py ${BENCH_ARGS:-} || exit $?
exit 0
