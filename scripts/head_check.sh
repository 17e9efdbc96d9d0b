set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/hc
echo "== pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/hc/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/hc/pytest.log
[ $rc -gt 1 ] && exit $rc
echo "== bench $(date +%T)"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/hc/bench.log 2>&1 || exit $?
tail -c 3000 gpurun_out/hc/bench.log
echo "== uncached-U bisect $(date +%T)"
timeout -k 10 400 python -u tools/uncached_u_bisect.py ${BISECT_CASES:-} > gpurun_out/hc/bisect.log 2>&1
rc=$?; cat gpurun_out/hc/bisect.log | grep -v amdgpu.ids; exit $rc
