#!/bin/bash
# Round 3: config 3's own counter record, then the multi-rank probes (virtual shards on one GPU).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 ./tools/msweep64_probe > gpurun_out/r03_msweep64_probe.txt 2>&1 || exit $?
mkdir -p gpurun_out
PROF_OUT=gpurun_out/prof3 PROF_ARGS="--gpus 1 --config config3 --secondary= --steps 20 --warmup 5 --no-update-bench" \
    bash scripts/profile.sh > gpurun_out/r03_prof3.log 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/p2p_probe.py config3 640 > gpurun_out/r03_multirank_config3.txt 2>&1 && \
timeout -k 10 400 python3 -u tools/p2p_probe.py config5 320 > gpurun_out/r03_multirank_config5.txt 2>&1
