# Whole -m gpu suite, smoke() and the driver's bench command on this tree (each under its own limit).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/hc
echo "== pytest $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/hc/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/hc/pytest.log
[ $rc -gt 1 ] && exit $rc
echo "== smoke $(date +%T)"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/hc/smoke.log 2>&1 || exit $?
tail -2 gpurun_out/hc/smoke.log
echo "== bench $(date +%T)"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/hc/bench.log 2>&1 || exit $?
grep '^{' gpurun_out/hc/bench.log | cut -c1-600
exit $rc
