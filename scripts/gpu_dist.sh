#!/bin/bash
# RCCL path on a 1-GPU box: the exchange kernels + real RCCL calls with a 1-rank communicator.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29512 scripts/dist_selftest.py --force-rccl > gpurun_out/dist1.log 2>&1
rc=$?; echo "dist1 rc=$rc"; grep -v amdgpu.ids gpurun_out/dist1.log | grep -v "^\[W" | tail -12
exit $rc
