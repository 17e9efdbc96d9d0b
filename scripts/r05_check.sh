#!/bin/bash
# Round-5 check on the GPU box: the new replicated-objective tests first, the whole GPU suite, then
# the multi-rank probe with the split and the replicated objective (config 3, virtual shards).
# Each step under its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${CHECK_TAG:-check}
mkdir -p $O
step() {
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; grep -v amdgpu.ids "$O/$name.log" | tail -${TAILN:-3} | cut -c1-300
    return $rc
}
step repl 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k replicated || exit $?
if [ "${SKIP_SUITE:-0}" != 1 ]; then
  step pytest 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread || exit $?
fi
TAILN=12 step p2p_repl 300 python -u tools/p2p_probe.py config3 640 --repl || exit $?
