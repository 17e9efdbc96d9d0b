#!/bin/bash
# Round 3: two-stage (64-pivot) peer-memory multi-rank batches (roles in separate loops, the first
# stage's U / F operands read with system-scope loads after a system-scope release at the switch):
# the whole -m gpu suite, then the multi-rank probes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03_pytest_gpu_v33.txt 2>&1 || exit $?
timeout -k 10 400 python3 -u tools/p2p_probe.py config3 640 > gpurun_out/r03_multirank_config3_v33.txt 2>&1 && \
timeout -k 10 400 python3 -u tools/p2p_probe.py config5 320 > gpurun_out/r03_multirank_config5_v33.txt 2>&1
