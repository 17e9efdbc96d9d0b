#!/bin/bash
# A round's final measurements: rocprofv3 profiles of the driver's bench command (scripts/profile_round.sh),
# then the plain driver command and the default bench.py run, each under its own limit.  Summaries are made in
# the build container from gpurun_out/$TAG (scripts/profile_bench.py, tools/pmc_summary.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-prof}
mkdir -p $O
PROF_OUT=$O bash scripts/profile_round.sh || exit $?
echo "== bench (driver's command) ($(date +%T))"
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || exit $?
tail -1 $O/bench_driver.log | cut -c1-300
echo "== bench (defaults) ($(date +%T))"
timeout -k 10 400 python3 bench.py > $O/bench_default.log 2>&1 || exit $?
tail -1 $O/bench_default.log | cut -c1-300
