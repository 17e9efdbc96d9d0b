source scripts/gpu_step.sh
SIMPLEX_POLL_WAVES=8 step parity 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "fused or batched or two_phase or config5_pivots or history or leaves_twice or hang" || exit $?
for v in 1 8 1 8; do SIMPLEX_POLL_WAVES=$v step stamps_$v 300 python -u tools/block_stamps.py config5,config3 || exit $?; grep -h "us:" $O/stamps_$v.log; done
TAG=${TAG}_ab REPS=2 VARIANTS="w1= w8=SIMPLEX_POLL_WAVES=8" bash scripts/ab.sh
