#!/bin/bash
# Round-2 closing run on one MI355X: the multi-rank paths on virtual shards (tools/p2p_probe.py,
# configs 3 and 5), then every -m gpu test, smoke and the driver's bench command
# (scripts/gpu_check.sh).  Each GPU step has its own time limit; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in config3 config5; do
  echo "== p2p probe $c ($(date +%T))"
  timeout -k 10 300 python -u tools/p2p_probe.py $c 320 > gpurun_out/p2p_$c.log 2>&1 || { tail -20 gpurun_out/p2p_$c.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/p2p_$c.log
done
BENCH_ARGS="--gpus 1 --steps 20 --warmup 5" bash scripts/gpu_check.sh
