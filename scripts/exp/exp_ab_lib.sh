#!/bin/bash
# Same-box A/B of the current library against ablib/libsimplex_prev.so (an earlier build, loaded
# through SIMPLEX_LIB_PATH): parity subset of the current one, per-block stamps and the driver's
# bench command of both.  (experiment helper)
source "$(dirname "$0")/../gpu_step.sh"
PREV=$(pwd)/ablib/libsimplex_prev.so
step parity 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -x -q -p no:cacheprovider --timeout 250 --timeout-method thread -k "${PK:-(fused or batched or two_phase or config5_pivots or history or leaves_twice or hang or published or virtual or replicated) and not long_pins and not whole_solve}" || exit $?
for v in new prev new prev; do
  if [ $v = prev ]; then export SIMPLEX_LIB_PATH=$PREV; else unset SIMPLEX_LIB_PATH; fi
  step stamps_$v 300 python -u tools/block_stamps.py config5,config3 || exit $?
  grep -h "us:" $O/stamps_$v.log
done
unset SIMPLEX_LIB_PATH
TAG=${TAG}_ab REPS=${REPS:-2} VARIANTS="new= prev=SIMPLEX_LIB_PATH=$PREV" bash scripts/ab.sh
