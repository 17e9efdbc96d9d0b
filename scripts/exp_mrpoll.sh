source scripts/gpu_step.sh
step parity 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "fused or batched or two_phase or config5_pivots or history or leaves_twice or hang or published" || exit $?
SIMPLEX_MR_POLLB=1 step mrparity 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_empty_shards.py tests/test_gpu_multigpu_mode.py -x -q -p no:cacheprovider --timeout 250 --timeout-method thread -k "p2p or replicated or virtual or multigpu or empty or unchanged or W" || exit $?
for v in 0 1 0 1; do SIMPLEX_MR_POLLB=$v step probe3_$v 200 python -u tools/p2p_probe.py config3 640 --repl || exit $?; done
for v in 0 1; do SIMPLEX_MR_POLLB=$v step probe5_$v 300 python -u tools/p2p_probe.py config5 640 --repl || exit $?; done
for f in $O/probe*.log; do echo "== $f"; grep -h "pivots/s" $f; done
