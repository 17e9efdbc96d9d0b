set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/exp1
for lay in 1 0; do for nl in 0 1; do
  echo "== blocked=$lay noleave=$nl"
  if [ $nl = 1 ]; then export SIMPLEX_BENCH_NOLEAVE=1; else unset SIMPLEX_BENCH_NOLEAVE; fi
  SIMPLEX_BLOCKED=$lay timeout -k 10 120 python -u tools/update_bench_probe.py 4096 8192 32 64 || exit 1
  SIMPLEX_BLOCKED=$lay timeout -k 10 120 python -u tools/update_bench_probe.py 16384 8192 32 || exit 1
done; done
