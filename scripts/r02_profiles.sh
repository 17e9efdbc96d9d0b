#!/bin/bash
# Round-2 profiles on the GPU box: rocprofv3 kernel trace + HBM counter passes of the driver's
# bench command (config 5, published as the bench's traffic record) and of a config-3 primary
# run (its secondary line's record), then the driver's bench command itself.  Every GPU step
# has its own time limit; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02_v2}
PROF_OUT=gpurun_out/prof5 bash scripts/profile.sh || exit 1
python3 scripts/profile_bench.py gpurun_out/prof5 ${TAG}_config5 5 20 "python3 bench.py --gpus 1 --steps 20 --warmup 5" --publish config5 > gpurun_out/prof5_summary.json || exit 1
C3="--config config3 --steps 278 --warmup 2 --secondary= --full-solves= --no-update-bench --no-cpu-baseline"
PROF_OUT=gpurun_out/prof3 PROF_ARGS="$C3" bash scripts/profile.sh || exit 1
python3 scripts/profile_bench.py gpurun_out/prof3 ${TAG}_config3 2 278 "python3 bench.py $C3" --publish config3 > gpurun_out/prof3_summary.json || exit 1
echo "== bench ($(date +%T))"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_${TAG}.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}.log | cut -c1-400
# (gpurun brings back only gpurun_out/: the summaries written into profiles/ travel that way)
mkdir -p gpurun_out/profiles_out
cp profiles/${TAG}_* profiles/pmc_sweep_config5.json profiles/pmc_sweep_config3.json gpurun_out/profiles_out/
cp gpurun_out/prof5/kt.log gpurun_out/profiles_out/${TAG}_config5_bench_under_rocprof.log
