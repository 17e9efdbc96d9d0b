set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider -k "p2p" > gpurun_out/pytest_p2p.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_p2p.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; exit $rc
