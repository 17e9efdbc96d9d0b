set -u
cd $GRAFT_REPO_ROOT
SWEEP_BATCH=32 SWEEP_RB=1,2,4 SWEEP_SC1=0,1 SWEEP_LDS=0,1 timeout -k 10 300 python tools/sweep_update.py config3 128 3 > gpurun_out/sweep.log 2>&1; cat gpurun_out/sweep.log
