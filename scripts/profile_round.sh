#!/bin/bash
# Profiles of the final code of a round: rocprofv3 kernel trace + HBM counters (FETCH_SIZE / WRITE_SIZE
# in passes of their own) + SQ counters of the driver's bench command (config 5), the same for
# config 3 alone, and the HBM counters of the synthetic update bench.  Each step under its own time
# limit; a failure ends the script.  Summaries: scripts/profile_bench.py, tools/pmc_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${PROF_OUT:-gpurun_out/prof}
mkdir -p $O
step() {
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -2 "$O/$name.log" | cut -c1-300
    return $rc
}
B5="--gpus 1 --steps 20 --warmup 5"
step kt 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py $B5 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  step $c 200 rocprofv3 --pmc $c --output-format csv -d $O/$c -o run -- python3 bench.py $B5 --no-cpu-baseline --full-solves= || exit $?
done
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE"
step sq 200 rocprofv3 --pmc $SQ --output-format csv -d $O/sq -o run -- python3 bench.py $B5 --no-cpu-baseline --full-solves= --secondary= --no-update-bench || exit $?
B3="--gpus 1 --config config3 --secondary= --steps 20 --warmup 5 --no-update-bench --no-cpu-baseline --full-solves="
step c3_kt 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3/kt -o run -- python3 bench.py $B3 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  step c3_$c 200 rocprofv3 --pmc $c --output-format csv -d $O/c3/$c -o run -- python3 bench.py $B3 || exit $?
done
for sz in "4096 8192" "16384 8192"; do
  tag=$(echo $sz | tr ' ' x)
  for c in FETCH_SIZE WRITE_SIZE; do
    step ub_${tag}_$c 150 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/ub_${tag}_$c -o run -- python3 tools/update_bench_probe.py $sz 32 || exit $?
  done
done
