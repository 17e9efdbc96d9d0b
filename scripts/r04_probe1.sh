#!/bin/bash
# Round-4 first measurements on the GPU box (each GPU step under its own time limit; a crash,
# abort or timeout ends the script): counter list, MFMA edge semantics, the gather probe, the
# chain's stage stamps, config 5's [-100,100] variant end to end, counters on the sweep and the
# fused batch, the update kernel in and out of the Infinity Cache.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/p1
mkdir -p $O
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -4 "$O/$name.log" | cut -c1-400
    return $rc
}
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ] && exit "$1"; return 0; }
step counters 120 rocprofv3 -L; fatal $?
step mfma_edge 120 experiments/mfma_edge_probe || exit $?
step gather_c5 240 experiments/gather_probe 32768 12800 64 144 400 || exit $?
step gather_c3 120 experiments/gather_probe 4096 12304 8 32 400 || exit $?
step stamps 300 python -u tools/stage_stamps.py config5,config3 || exit $?
step blocks 300 python -u tools/block_stamps.py config5,config3 || exit $?
step variant 900 python -u tools/variant_solve.py --json $O/variant.json || exit $?
BENCH="bench.py --steps 20 --warmup 5 --no-cpu-baseline --full-solves= --secondary= --no-update-bench"
has() { for c in "$@"; do grep -qw "$c" $O/counters.log || return 1; done; return 0; }
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE"
if has $SQ; then
  step pmc_sq 240 timeout -s KILL 200 rocprofv3 --pmc $SQ --output-format csv -d $O/pmc_sq -o run -- python3 $BENCH || exit $?
else echo "skip pmc_sq: counters missing"; fi
TCP=""
for c in TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_PERMISSION_MISS_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum; do
  has $c && TCP="$TCP $c"
done
if [ -n "$TCP" ]; then
  step pmc_tcp 240 timeout -s KILL 200 rocprofv3 --pmc $TCP --output-format csv -d $O/pmc_tcp -o run -- python3 $BENCH || exit $?
else echo "skip pmc_tcp: counters missing"; fi
for sz in "4096 8192" "8192 8192" "16384 8192"; do
  tag=$(echo $sz | tr ' ' x)
  step ub_$tag 180 python -u tools/update_bench_probe.py $sz 32 64 || exit $?
  for c in FETCH_SIZE WRITE_SIZE; do
    step ub_${tag}_$c 180 timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/ub_${tag}_$c -o run -- python3 tools/update_bench_probe.py $sz 32 || exit $?
  done
done
exit 0
