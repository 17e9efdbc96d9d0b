# Round 5: the separate leaving-row fix-up (SIMPLEX_SEP_FIXUP=1, k_mfixup) -- parity files under the
# switch, then a same-box A/B of the driver's bench command against the default.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/sep
echo "== parity (sep) $(date +%T)"
SIMPLEX_SEP_FIXUP=1 timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/sep/parity.log 2>&1
rc=$?; tail -3 gpurun_out/sep/parity.log; [ $rc -ne 0 ] && exit $rc
TAG=sep REPS=3 VARIANTS="base= sep=SIMPLEX_SEP_FIXUP=1" bash scripts/r05_ab.sh
