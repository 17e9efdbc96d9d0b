#!/bin/bash
# rocprofv3 passes over the driver's own bench command: kernel trace + stats, then the HBM
# counters in passes of their own (FETCH_SIZE and WRITE_SIZE cannot share one pass on gfx950).
# The PMC passes skip the CPU baseline and the full solves (no sweeps of the primary workload
# there; they only lengthen the run).  Summaries: python scripts/profile_bench.py (see there).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/prof}
mkdir -p $OUT
ARGS=${PROF_ARGS:---gpus 1 --steps 20 --warmup 5}
echo "== kernel trace: bench.py $ARGS ($(date +%T))"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py $ARGS > $OUT/kt.log 2>&1 || { echo "kt failed"; tail -20 $OUT/kt.log; exit 1; }
tail -1 $OUT/kt.log
for c in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $c ($(date +%T))"
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- python3 bench.py $ARGS --no-cpu-baseline --full-solves= > $OUT/$c.log 2>&1 || { echo "pmc $c failed"; tail -20 $OUT/$c.log; exit 1; }
  tail -1 $OUT/$c.log | cut -c1-200
done
