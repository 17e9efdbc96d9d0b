#!/bin/bash
# GPU-call helpers: each step under its own time limit, its log under gpurun_out/$TAG; a failure
# ends the calling script (source this file, then `step NAME SECONDS CMD...`).
set -u
cd "${GRAFT_REPO_ROOT:-$(git -C "$(dirname "$0")" rev-parse --show-toplevel 2>/dev/null || echo "$(dirname "$0")/..")}"
export TMPDIR=/tmp
TAG=${TAG:-run}
O=gpurun_out/$TAG
mkdir -p "$O"
step() {
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -${TAILN:-6} "$O/$name.log" | cut -c1-400
    return $rc
}
