#!/bin/bash
# Round-4 development loop on the GPU box: the GPU test suite (or a subset: PYTEST_ARGS), the
# chain's stage and block stamps, a short bench of configs 5 and 3.  Each GPU step under its own
# time limit; a failing test run, crash, abort or timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${ITER_TAG:-it}
mkdir -p $O
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -${TAILN:-4} "$O/$name.log" | cut -c1-400
    return $rc
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} || exit $?
fi
step stamps 300 python -u tools/stage_stamps.py config5,config3 || exit $?
step blocks 300 python -u tools/block_stamps.py config5,config3 || exit $?
step bench 600 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --full-solves= --no-update-bench || exit $?
python3 - "$O/bench.log" <<'EOF'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith('{')][-1]
d = json.loads(line)
pr = d['config']['per_rank'][0]
print(f"config5 {d['value']:.0f} pivots/s  us/pivot {pr['us_per_pivot']:.2f} sweep {pr['sweep_us_per_pivot']:.2f} chain {pr['chain_us_per_pivot']:.2f}  frac {d['roofline']['frac']:.3f}")
s = d.get('secondary')
if s:
    print(f"config3 {s['value']:.0f} pivots/s  ms/step {s['ms_per_step']:.3f}  frac {s['roofline']['frac']:.3f}")
EOF
exit 0
