#!/bin/bash
# Development loop on the GPU box: parity tests, then a kernel-trace profile of a short bench
# run and its per-pivot breakdown.  Each GPU step has its own time limit; any failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
rm -rf gpurun_out/it
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/it -o run -- python3 bench.py ${ITER_ARGS:---steps 2000 --warmup 50 --no-cpu-baseline --secondary= --update-events 0} > gpurun_out/it.log 2>&1 || { tail -20 gpurun_out/it.log; exit 1; }
tail -1 gpurun_out/it.log | cut -c1-600
python3 scripts/chain_stats.py gpurun_out/it/run_kernel_trace.csv
