# Round-5 bisect of the uncached-U divergence: TREES = directories holding an older
# commit's built package + tools/uncached_u_bisect.py; then the empty-shard tests and the bisect on this tree.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/ob
for o in ${TREES:-}; do
  echo "== $o $(date +%T)"
  (cd $o && BISECT_REPS=${REPS:-5} timeout -k 10 300 python -u tools/uncached_u_bisect.py ${CASES:-unc}) > gpurun_out/ob/$o.log 2>&1
  rc=$?; echo "OK lines: $(grep -c OK gpurun_out/ob/$o.log)"; grep MISMATCH gpurun_out/ob/$o.log; [ $rc -ne 0 ] && exit $rc
done
echo "== empty-shard tests $(date +%T)"
timeout -k 10 300 python -u -m pytest tests/test_gpu_empty_shards.py -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ob/empty_tests.log 2>&1
rc=$?; tail -12 gpurun_out/ob/empty_tests.log; [ $rc -ne 0 ] && exit $rc
echo "== HEAD bisect $(date +%T)"
BISECT_REPS=${REPS:-5} timeout -k 10 300 python -u tools/uncached_u_bisect.py unc,unc_p2p > gpurun_out/ob/head_pooled.log 2>&1
rc=$?; echo "OK lines: $(grep -c OK gpurun_out/ob/head_pooled.log)"; grep MISMATCH gpurun_out/ob/head_pooled.log; exit $rc
