#!/bin/bash
# rocprofv3 passes over a short bench run: kernel trace + stats, then HBM counters in their
# own passes (FETCH_SIZE and WRITE_SIZE cannot share one pass on gfx950).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS=${PROF_ARGS:---steps 2000 --warmup 64 --no-cpu-baseline --secondary= --no-full-solve --update-events 0}
echo "== kernel trace ($(date +%T))"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py $ARGS > $OUT/kt.log 2>&1 || { echo "kt failed"; tail -20 $OUT/kt.log; exit 1; }
tail -2 $OUT/kt.log
for c in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $c ($(date +%T))"
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- python3 bench.py $ARGS > $OUT/$c.log 2>&1 || { echo "pmc $c failed"; tail -20 $OUT/$c.log; exit 1; }
  tail -1 $OUT/$c.log
done
find $OUT -name "*.csv" | head -20
