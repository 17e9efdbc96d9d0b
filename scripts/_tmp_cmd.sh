set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider -k "p2p or batched or config2 or published or large_batch or same_row" > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/batch_stamps.py config3 20 32 > gpurun_out/stamps3.log 2>&1; cat gpurun_out/stamps3.log
timeout -k 10 200 python tools/batch_stamps.py config5 10 32 > gpurun_out/stamps5.log 2>&1; cat gpurun_out/stamps5.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b.log 2>&1 || exit 1
python3 -c "import json; r=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]); print(round(r['value']), r['roofline']['frac'], round(r['secondary']['value']))"
