#!/bin/bash
# Round-4 second measurements (each GPU step under its own limit; a crash, abort or timeout ends
# the script): the gather probe with blocked layouts and pollers, config 5's [-100,100] variant,
# counters on the sweep / fused batch, the f64 ceiling with its clock, the update kernel in and
# out of the Infinity Cache, the r03 records DESIGN cites (MFMA probe, uncached bisect + reuse).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/p2
mkdir -p $O
step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -3 "$O/$name.log" | cut -c1-300
    return $rc
}
step gather_c5 240 experiments/gather_probe 32768 12800 64 144 300 144 || exit $?
step mfma_f64_probe 60 experiments/mfma_f64_probe || exit $?
step variant 900 python -u tools/variant_solve.py --json $O/variant.json || exit $?
BENCH="bench.py --steps 20 --warmup 5 --no-cpu-baseline --full-solves= --secondary= --no-update-bench"
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE"
step pmc_sq 240 timeout -s KILL 200 rocprofv3 --pmc $SQ --output-format csv -d $O/pmc_sq -o run -- python3 $BENCH || exit $?
TCP="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_PERMISSION_MISS_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"
step pmc_tcp 240 timeout -s KILL 200 rocprofv3 --pmc $TCP --output-format csv -d $O/pmc_tcp -o run -- python3 $BENCH || exit $?
step f64_rate 120 timeout -s KILL 100 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 --kernel-trace --output-format csv -d $O/f64_rate -o run -- experiments/f64_rate_probe || exit $?
for sz in "4096 8192" "8192 8192" "16384 8192"; do
  tag=$(echo $sz | tr ' ' x)
  step ub_$tag 180 python -u tools/update_bench_probe.py $sz 32 64 || exit $?
  for c in FETCH_SIZE WRITE_SIZE; do
    step ub_${tag}_$c 180 timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/ub_${tag}_$c -o run -- python3 tools/update_bench_probe.py $sz 32 || exit $?
  done
done
step reuse 120 experiments/uncached_reuse_probe || exit $?
step reuse_wb 120 experiments/uncached_reuse_probe --writeback || exit $?
for mode in 0 1 2 3; do
  step bisect_$mode 300 python -u experiments/uncached_exchange_probe.py $mode || exit $?
done
exit 0
