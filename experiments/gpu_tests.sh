#!/bin/bash
# GPU-box test run: the given pytest selection (default: every -m gpu test), then optional
# in-kernel stamp profiles of the fused batch.  Each GPU step has its own time limit; a crash,
# abort or timeout ends the script (a plain test failure, exit 1, does not).
#   TESTS="tests/test_x.py ..." STAMPS=1 bash scripts/gpu_tests.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== pytest ${TESTS:-tests} ($(date +%T))"
timeout -k 10 1500 python -u -m pytest ${TESTS:-tests} -m gpu -q --maxfail=10 -p no:cacheprovider \
    --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "== pytest rc=$rc"
tail -15 gpurun_out/pytest_gpu.log
[ $rc -gt 1 ] && exit $rc
if [ "${STAMPS:-0}" = "1" ]; then
  for c in config5 config3; do
    echo "== stamps $c ($(date +%T))"
    timeout -k 10 200 python -u tools/batch_stamps.py $c 10 32 > gpurun_out/stamps_$c.log 2>&1 || exit $?
    cat gpurun_out/stamps_$c.log
  done
fi
exit $rc
