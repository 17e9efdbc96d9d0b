#!/bin/bash
# Round-2 check of the sweep-written timing records (no device copies between the kernels of a
# bench session's timed region): the session tests, the driver's bench command, and its kernel
# trace (per-batch timeline).  Each GPU step has its own time limit; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== pytest ($(date +%T))"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -m gpu -q -x -p no:cacheprovider \
    --timeout 300 --timeout-method thread -k "session or negated or width or virtual or large or p2p" \
    > gpurun_out/pytest_rec.log 2>&1 || { tail -30 gpurun_out/pytest_rec.log; exit 1; }
tail -2 gpurun_out/pytest_rec.log
echo "== bench ($(date +%T))"
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_rec.log 2>&1 || { tail -20 gpurun_out/bench_rec.log; exit 1; }
tail -1 gpurun_out/bench_rec.log | cut -c1-300
echo "== kernel trace ($(date +%T))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rec -o run -- python3 bench.py \
    --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --full-solves= --secondary= --no-update-bench > gpurun_out/prof_rec.log 2>&1 \
    || { tail -20 gpurun_out/prof_rec.log; exit 1; }
tail -1 gpurun_out/prof_rec.log | cut -c1-300
