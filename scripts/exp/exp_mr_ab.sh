#!/bin/bash
# Same-box A/B of the multi-rank (virtual peer-memory ranks) chain: the current library against
# ablib/libsimplex_prev.so, tools/p2p_probe.py per config, split and replicated objective.
# (experiment helper)
source "$(dirname "$0")/../gpu_step.sh"
PREV=$(pwd)/ablib/libsimplex_prev.so
if [ -n "${PK:-}" ]; then
  step parity 700 python -u -m pytest ${FILES:-tests} -x -q -p no:cacheprovider --timeout 250 --timeout-method thread -m gpu -k "$PK" || exit $?
  tail -1 $O/parity.log
fi
for v in new prev new prev; do
  if [ $v = prev ]; then export SIMPLEX_LIB_PATH=$PREV; else unset SIMPLEX_LIB_PATH; fi
  for cfg in config3 config5; do
    step p2p_${cfg}_$v 300 python -u tools/p2p_probe.py $cfg 640 --repl || exit $?
    echo "-- $v $cfg"; tail -12 $O/p2p_${cfg}_$v.log
  done
done
