"""Benchmark: simplex pivots/s and HBM GB/s of the rank-1 tableau update on MI355X.

Workload (BASELINE.json configs[4], the m=32768 problem north_star's scaling target is
quoted on): generateRandomProblem(n=8192, m=32768, seed=851968, [1,100]) -- seed n*100+m as
the reference's -t sweep (main.cu:56-64) -- phase-1 tableau 32768 x 73729 fp64, synthesised
in HBM (10.7 GB stored: artificial columns aliased to their slack columns).
A "step" is one pass of the hot path over the tableau: one batch of simplex pivots (64: two
stages of 32, DESIGN.md §3, on one GPU and on several) -- entering argmin, ratio test,
pivot row and objective row of each -- followed by one sweep that applies their rank-1 updates
to every stored tableau element.  W untimed steps, then K timed steps: by default the driver's
window, W = 5 and K = 20 (phase-1 pivots 320..1600 of the first 2000), whose end
state is checked against the CPU oracle's pin at pivot 1600 (the line's `parity`); --steps 0 times
up to about pivot 2080.  Every timed step is a full batch, so the timed window runs exactly the kernels
the warmup ran.

N GPUs: the constraint rows are split into N contiguous 512-aligned blocks, each GPU sweeps only
its rows; per pivot the shards exchange the tile winners and the pivot row (peer memory over
xGMI inside one launch per GPU per batch, or per-pivot collectives).  Two launch forms:
  * torchrun (WORLD_SIZE > 1; the driver's form): one process per GPU, RCCL communicator;
  * `python bench.py --gpus N` without torchrun: ONE process drives GPUs 0..N-1 through the
    library's SIMPLEX_GPUS mode (the drop-in's own multi-GPU form); it exits
    non-zero when fewer than N GPUs are visible.
The problem is the same at every N ("strong" scaling).

Secondary (same JSON line): config 3, the reference's own 8192 x 4096 -t instance, whose
4096-row tableau the roofline target is quoted on (8900 of its 8981 phase-1 pivots, with
its own sweep roofline), and at N=1 its end-to-end twoPhaseMethod solve.

The CPU baseline is the serial C oracle (oracle/, a restatement of the reference's
algorithm -- the reference has no CPU path) on the first pivots of the primary instance,
pinned to one core; the same pivots are re-run on the GPU and checked bit for bit.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (n, m, seed) -- seed n*100+m as main.cu:63, values in [+1,+100] (main.cu:64)
    "config2": (2048, 1024, 205824),
    "config3": (8192, 4096, 823296),
    "config4": (4096, 16384, 425984),
    "config5": (8192, 32768, 851968),
}
# oracle pivots timed for the CPU baseline (first 50 / 10 / 3 pivots)
CPU_SAMPLE = {"config2": 200, "config3": 50, "config4": 10, "config5": 5}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
F64_SPEC_TFLOPS = 78.6  # MI355X fp64 matrix (= vector) spec peak
# the fp64 matrix rate this chip sustains: v_mfma_f64_16x16x4f64 alone on every SIMD, 2-4 waves each
# (experiments/f64_rate_probe.hip, profiles/r03_f64_rate_probe.txt: 46.8-47.6 TFLOP/s)
F64_MFMA_MEASURED_TFLOPS = 47.6
# reference: RTX 2070 Super, config 3 phase 1, mean 7607.5 us per pivot
REF_PIVOTS_PER_S = {"config3": 1e6 / 7607.5}  # (no published number for configs 4-5)
# reference: RTX 2070 Super, config 3, pivot-loop totals 68.33 s (phase 1) + 0.94 s (phase 2), 8981 + 255 pivots
REF_SOLVE = {"config3": {"pivot_loop_s": 68.33 + 0.94, "pivots": [8981, 255]}}


def _sha(a):
    import hashlib

    import numpy as np
    return hashlib.sha256(memoryview(np.ascontiguousarray(a)).cast("B")).hexdigest()


def _golden(name):
    path = os.path.join(ROOT, "tests", "golden", name)
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        return json.load(f)


def window_parity(config, pivots, d, base):
    """The timed run's own end state against the CPU oracle's pin at the same pivot count
    (tests/golden/long_pivots.json, tests/golden/scripts/make_long_pins.py): d[0]'s bits and the
    SHA-256 of the objective row and the basis (the tableau's digest is checked by
    tests/test_gpu_large.py); None when no pin sits at this pivot count."""
    rec = _golden("long_pivots.json").get(config)
    if not rec:
        return None
    pin = [c for c in rec["checkpoints"] if c.get("phase", 1) == 1 and c["pivots"] == pivots]
    if not pin:
        return None
    pin = pin[0]
    ok = {"d0_bits": float(d[0]).hex() == pin["d0_hex"], "objective_row_sha256": _sha(d) == pin["sha256_d"],
          "basis_sha256": _sha(base) == pin["sha256_base"]}
    return {"pivots": pivots, "oracle_pin": f"tests/golden/long_pivots.json[{config}] at pivot {pivots}",
            "match": all(ok.values()), **ok}


def solve_parity(name, res):
    """A whole twoPhaseMethod against the CPU oracle's whole-solve pin (status, pivot counts, the
    objective's bits, SHA-256 of basis and solution), where one exists."""
    pin = _golden("oracle_solves.json").get(name)
    src = "tests/golden/oracle_solves.json"
    if pin is None:
        r = (_golden("long_pivots.json").get(name) or {}).get("result")
        if r and "opt_hex" in r:
            pin = {"status": r["status"], "pivots": r["pivots"], "opt_hex": r["opt_hex"],
                   "base_sha256": r["sha256_base"], "x_sha256": r["sha256_x"]}
            src = "tests/golden/long_pivots.json"
    if pin is None:
        return None
    import numpy as np
    ok = {"status": res.status == pin["status"], "pivots": list(res.pivots) == list(pin["pivots"]),
          "objective_bits": float(res.optimal_value).hex() == pin["opt_hex"],
          "basis_sha256": _sha(np.asarray(res.base, dtype=np.int32)) == pin["base_sha256"],
          "solution_sha256": _sha(np.asarray(res.solution, dtype=np.float64)) == pin["x_sha256"]}
    return {"oracle_pin": f"{src}[{name}]", "match": all(ok.values()), **ok}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(n, m, seed, pivots, sx):
    """Time the serial oracle on the first `pivots` phase-1 pivots (one pinned core) and
    check the GPU reproduces the same pivots bit for bit."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np

    import oracle

    A, b, c = oracle.generate(n, m, seed, 1, 100)
    T, d, base = oracle.build_phase1(A, b)
    oracle.update_objective(T, d, base)
    T_gpu, d_gpu, base_gpu = T.copy(), d.copy(), base.copy()
    old = os.sched_getaffinity(0)
    core = min(old)
    os.sched_setaffinity(0, {core})
    try:
        t0 = time.perf_counter()
        st, done = oracle.solve(T, d, base, max_pivots=pivots)
        dt = time.perf_counter() - t0
    finally:
        os.sched_setaffinity(0, old)
    sx.dev_pivots(T_gpu, d_gpu, base_gpu, pivots)
    same = (np.array_equal(T.view(np.uint64), T_gpu.view(np.uint64))
            and np.array_equal(d.view(np.uint64), d_gpu.view(np.uint64))
            and np.array_equal(base, base_gpu))
    N1 = 1 + n + 2 * m
    return {
        "value": done / dt,
        "unit": "pivots/s",
        "cores": 1,
        "kind": "port",
        "sample": f"first {done} phase-1 pivots of the same instance ({m}x{N1} fp64 tableau), serial C oracle",
        "seconds": dt,
        "update_GBps": 16.0 * (m + 1) * N1 * done / dt / 1e9,
        "cpu_model": cpu_model(),
        "core_used": core,
        "host_cores_total": os.cpu_count(),
        "gpu_bit_exact_on_sample": bool(same),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20,
                    help="timed steps; a step = one batch of pivots + one tableau sweep (0 = up to about pivot 2080)")
    ap.add_argument("--warmup", type=int, default=5, help="untimed steps before timing")
    ap.add_argument("--config", default="config5", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0,
                    help="pivots per tableau sweep (0 = library default: 64 from 4096 rows, else 32)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--update-events", type=int, default=1,
                    help="bracket every k-th sweep launch with HIP events (0 = none)")
    ap.add_argument("--pmc-dir", default=os.path.join(ROOT, "profiles"),
                    help="directory of pmc_sweep_<config>.json: per-launch HBM bytes of the sweep (rocprofv3 --pmc)")
    ap.add_argument("--secondary", default="config3",
                    help="second workload timed in the same run ('' to skip): the roofline-target tableau")
    ap.add_argument("--secondary-steps", type=int, default=0,
                    help="config 3 (0 = up to pivot 8960 of its 8981 phase-1 pivots)")
    ap.add_argument("--secondary-warmup", type=int, default=2)
    ap.add_argument("--full-solves", default="config3,config4,config5",
                    help="instances solved end to end by twoPhaseMethod at N=1 ('' to skip)")
    ap.add_argument("--no-update-bench", action="store_true",
                    help="skip the synthetic 4096x8192 sweep bench (SURVEY.md §8d config 3')")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.gpus not in (1, world):
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} processes", file=sys.stderr)
        sys.exit(2)
    single_process_gpus = world == 1 and args.gpus > 1
    if single_process_gpus:
        visible = torch.cuda.device_count()  # (counts devices without initialising them)
        if visible < args.gpus:
            print(f"bench.py: --gpus {args.gpus} needs {args.gpus} GPUs, {visible} visible", file=sys.stderr)
            sys.exit(2)
    n_gpus = world if world > 1 else max(args.gpus, 1)
    torch.cuda.set_device(local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    import simplexoncuda_amd as sx
    from simplexoncuda_amd import dist as sxdist

    if world > 1:
        sxdist.init_from_torch(local_rank)
    else:
        sx.load().simplex_set_device(local_rank)
        if single_process_gpus:
            sx.set_gpus(list(range(args.gpus)))
    sx.set_batch(args.batch)

    def barrier():
        if world > 1:
            dist.barrier()

    def measure(config, steps, warmup, events, last_pivot=2016 + 64):
        """W untimed + `steps` timed steps (batches of K pivots + one sweep) of `config`'s phase 1;
        steps = 0: up to pivot `last_pivot`."""
        n, m, seed = CONFIGS[config]
        t_setup = time.perf_counter()
        # generateRandomProblem(n, m, seed, 1, 100) synthesised directly in HBM, each rank its rows
        sess = sx.Session(generated=(n, m, seed, 1, 100))
        torch.cuda.synchronize()
        t_setup = time.perf_counter() - t_setup
        K = sess.batch()  # pivots per step: the library's batch on this engine
        if steps <= 0:
            steps = max(1, (last_pivot - warmup * K) // K)
        if warmup > 0:
            sess.pivots(warmup * K)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tim = sess.pivots(steps * K, time_updates=events)
        torch.cuda.synchronize()
        barrier()
        elapsed = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            elapsed = float(tt.item())
        parity = None
        if world == 1:  # (outside the timed region: the run's own end state vs the oracle's pin)
            d_end, base_end = sess.objective_row_and_basis(m, 1 + n + 2 * m)
            parity = window_parity(config, (warmup + steps) * K, d_end, base_end)
        # per-rank split of the pivot time: this rank's timed sweeps vs the rest (the chain: the
        # fused batches, slack exchanges and launch gaps), from its own HIP events
        mine = {"rank": rank, "rows": tim.local_rows, "pivots": tim.pivots,
                "us_per_pivot": tim.wall_ms * 1e3 / max(tim.pivots, 1),
                "sweep_us_per_pivot": tim.update_ms * 1e3 / max(tim.pivots, 1),
                "chain_us_per_pivot": (tim.wall_ms - tim.update_ms) * 1e3 / max(tim.pivots, 1)}
        if world > 1:
            per_rank = [None] * world
            dist.all_gather_object(per_rank, mine)
        else:
            per_rank = [mine]
        sess.close()
        avg_update_s = tim.update_ms / 1e3 / max(tim.update_launches, 1)
        # algorithmic bytes of a sweep: every stored tableau element it moves, read and written once
        achieved = tim.swept_bytes / (tim.update_ms / 1e3) / 1e9 if tim.update_launches else None
        return {"n": n, "m": m, "seed": seed, "tim": tim, "elapsed": elapsed, "pivots": tim.pivots,
                "avg_update_s": avg_update_s, "achieved": achieved, "setup_s": t_setup,
                "steps": steps, "warmup": warmup, "per_rank": per_rank, "K": K, "parity": parity}

    def roofline(cfg, r):
        tim, achieved = r["tim"], r["achieved"]
        traffic, source = None, None
        pmc = os.path.join(args.pmc_dir, f"pmc_sweep_{cfg}.json") if args.pmc_dir else None
        if pmc and os.path.exists(pmc):
            with open(pmc) as f:
                rec = json.load(f)
            traffic = rec.get("hbm_bytes_per_launch")
            source = (f"committed profile profiles/pmc_sweep_{cfg}.json ({rec.get('tag')}: rocprofv3 --pmc "
                      f"FETCH_SIZE and WRITE_SIZE passes of `{rec.get('command', 'bench.py')}`, "
                      "(2*FETCH_SIZE+WRITE_SIZE)*1024 per launch) -- not measured in this run")
        return {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS if achieved else None,
            "traffic": traffic,
            "traffic_source": source,
            "kernel": ("k_msweep<16> (the batch's 64 rank-1 pivot updates applied to the tableau on the matrix "
                       "cores, rank 0)" if r["K"] > 32 else
                       "k_sweep (the batch's rank-1 pivot updates applied to the tableau, rank 0)"),
            "bytes_definition": "16 * rows * (1 + n + touched slack columns) per sweep: every stored tableau "
                                "element the sweep moves, read and written once (SURVEY.md §8d 16(m+1)N over the "
                                "swept columns; artificial columns alias their slacks and untouched slack columns "
                                "are exact unit vectors, DESIGN.md §2, §3.4)",
            "algorithmic_bytes_per_launch": tim.update_bytes,
            "pivots_per_launch": tim.swept_pivots / max(tim.update_launches, 1),
            "avg_launch_us": r["avg_update_s"] * 1e6,
            "timed_launches": tim.update_launches,
            "timing": "HIP events on the engine stream around every timed sweep",
            "sweep_share_of_time": tim.update_ms / max(tim.wall_ms, 1e-9),
            "compute": compute_roof(tim),
        }

    def compute_roof(tim):
        """The sweep's fp64 work against the matrix-core rate: 2 flops per swept element per pending
        pivot.  A 64-slot sweep does 128 flops per 16 bytes moved, so it is co-bound by the fp64
        matrix rate."""
        if not tim.update_launches or tim.update_ms <= 0:
            return None
        flops = 2.0 * (tim.swept_pivots / tim.update_launches) * (tim.swept_bytes / 16.0)
        tf = flops / (tim.update_ms / 1e3) / 1e12
        return {"achieved_tflops": tf, "spec_peak_tflops": F64_SPEC_TFLOPS,
                "measured_mfma_ceiling_tflops": F64_MFMA_MEASURED_TFLOPS,
                "frac_of_spec": tf / F64_SPEC_TFLOPS, "frac_of_measured_ceiling": tf / F64_MFMA_MEASURED_TFLOPS,
                "ceiling_source": "profiles/r03_f64_rate_probe.txt (v_mfma_f64_16x16x4f64 on every SIMD, no memory)"}

    def exchange_name():
        if n_gpus == 1:
            return "none (one shard)"
        # the start-up self-check's verdict on these devices (simplex_multi_gpu_mode)
        mode = sx.load().simplex_multi_gpu_mode()
        form = "" if world > 1 else ", one launch per GPU"
        return {2: f"peer-memory fused batch{form} (xGMI)",
                1: ("per-pivot exchange (FALLBACK: the peer-memory batches failed the self-check against a "
                    "one-shard solve; slower than 1 GPU)"),
                0: ("none: every solve on one device (FALLBACK: the shards' exchange failed the self-check "
                    "against a one-shard solve)")}.get(mode, f"unknown (self-check not run, mode {mode})")

    def workload(cfg, r):
        return (f"{cfg}: phase-1 pivots, {r['m']}x{1 + r['n'] + 2 * r['m']} fp64 tableau "
                f"(m={r['m']}, n={r['n']}, seed={r['seed']})")

    r = measure(args.config, args.steps, args.warmup, args.update_events)
    n, m, seed, tim, elapsed, pivots = r["n"], r["m"], r["seed"], r["tim"], r["elapsed"], r["pivots"]
    K, steps = r["K"], r["steps"]
    out = {
        "metric": "simplex pivots/sec + HBM GB/s on gaussian update, dense m×n tableau",
        "value": pivots / elapsed,
        "unit": "pivots/s",
        "n_gpus": n_gpus,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / max(steps, 1),
        "ms_per_pivot": elapsed * 1e3 / max(pivots, 1),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": (pivots / elapsed) / REF_PIVOTS_PER_S[args.config] if args.config in REF_PIVOTS_PER_S else None,
        "dtype": "f64",
        "data": f"synthetic: generateRandomProblem(n={n}, m={m}, seed={seed}, [1,100]) -- seed n*100+m as the "
                "reference's -t sweep (cuRAND-XORWOW + MSVC rand semantics), synthesised on the GPU",
        "config": {
            "workload": workload(args.config, r),
            "step": f"one batch of {K} pivots + one sweep of the tableau",
            "pivots_per_step": K,
            "m": m, "n": n, "seed": seed, "tableau_width": tim.width, "stored_width": tim.stored_width,
            "rows_per_gpu_rank0": tim.local_rows, "parallelism": f"row-block x{n_gpus}",
            "launch": ("one process per GPU (torchrun, RCCL)" if world > 1 else
                       f"one process driving GPUs 0..{n_gpus - 1} (SIMPLEX_GPUS)" if single_process_gpus else
                       "one process, one GPU"),
            "exchange": exchange_name(),
            "per_rank": r["per_rank"],
            "pivots_timed": pivots, "first_timed_pivot": args.warmup * K, "status_after": tim.status,
            "setup_s": r["setup_s"],
        },
        "parity": r["parity"],
        "roofline": roofline(args.config, r),
        "cpu_baseline": None,
    }
    if args.secondary and args.secondary != args.config:
        r2 = measure(args.secondary, args.secondary_steps, args.secondary_warmup, args.update_events, last_pivot=8960)
        out["secondary"] = {
            "workload": workload(args.secondary, r2),
            "value": r2["pivots"] / r2["elapsed"], "unit": "pivots/s",
            "vs_baseline": (r2["pivots"] / r2["elapsed"]) / REF_PIVOTS_PER_S[args.secondary]
            if args.secondary in REF_PIVOTS_PER_S else None,
            "ms_per_step": r2["elapsed"] * 1e3 / max(r2["steps"], 1), "pivots_per_step": r2["K"],
            "steps": r2["steps"], "warmup": args.secondary_warmup, "pivots_timed": r2["pivots"],
            "first_timed_pivot": args.secondary_warmup * r2["K"],
            "status_after": r2["tim"].status, "rows_per_gpu_rank0": r2["tim"].local_rows, "setup_s": r2["setup_s"],
            "roofline": roofline(args.secondary, r2),
        }
    if n_gpus == 1 and not args.no_update_bench:
        # SURVEY.md §8d config 3': the sweep kernel alone on a synthetic 4096 x 8192 fp64 matrix
        # (uniform [1,100], seed 823296) with K random pending pivots, K = the pivot loop's batch
        # (three runs of 10 untimed + 50 timed sweeps each; the median run is reported -- the
        # first run on a box is often 5-10 % slower); the one-stage variants alongside
        def sweep_bench(pivots, mfma, rows=4096):
            sx.set_sweep_mfma(mfma)
            runs = [sx.bench_sweep(rows, 8192, 823296, 1, 100, pivots, warmup=10, iters=50) for _ in range(3)]
            sx.set_sweep_mfma(-1)
            us, nbytes = sorted(runs)[1]
            gbs = nbytes / (us * 1e-6) / 1e9
            return {"pivots_per_sweep": pivots,
                    "kernel": ("k_msweep<%d> (matrix cores)" % (pivots // 4 if pivots > 32 else 8)) if mfma or pivots > 32
                    else "k_sweep<32,4,1> (vector units)",
                    "runs_us": [x[0] for x in runs], "avg_launch_us": us, "bytes_per_launch": nbytes, "achieved": gbs,
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS, "us_per_pivot": us / pivots}
        # north_star's update-kernel target: the sweep of one 32-pivot batch (k_msweep<8>, the
        # one-stage kernel); the 64-pivot sweep the loop runs on >= 4096 rows and the vector
        # sweep alongside (the 64-pivot one moves half the bytes per pivot at a lower fraction of
        # peak: it is co-bound by the fp64 matrix rate)
        K3 = r["K"] if args.config == "config3" else (r2["K"] if args.secondary == "config3" else 32)
        variants = [sweep_bench(32, 1), sweep_bench(64, 1), sweep_bench(32, 0)]
        # the same kernel on a matrix 8x the Infinity Cache (2.1 GB): every byte from HBM
        big = sweep_bench(32, 1, rows=16384)
        big["workload"] = "16384x8192 (2.1 GB, 8x the 256 MiB Infinity Cache), 32 pivots per sweep"
        pmc_ub = os.path.join(args.pmc_dir, "pmc_update_bench.json") if args.pmc_dir else None
        ub_traffic = None
        if pmc_ub and os.path.exists(pmc_ub):
            with open(pmc_ub) as f:
                ub_traffic = json.load(f)
        out["update_bench"] = dict(variants[0], workload=(
            "config3': the 32-pivot sweep kernel on a synthetic 4096x8192 fp64 matrix (uniform [1,100], seed "
            "823296) with 32 random pending pivots (distinct pseudo-random leaving rows since round 5), median of 3 "
            "runs of 50 timed sweeps (HIP events)"),
            note="the matrix (268 MB) is about the size of the 256 MB Infinity Cache, so sweeps partly hit it; "
                 "out_of_cache is the same kernel on a 2.1 GB matrix (HBM rate)",
            traffic=(ub_traffic or {}).get("4096x8192"),
            traffic_source=("committed profile profiles/pmc_update_bench.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                            "passes of tools/update_bench_probe.py, (2*FETCH_SIZE+WRITE_SIZE)*1024 per launch; FETCH_SIZE "
                            "counts Infinity-Cache hits too) -- not measured in this run") if ub_traffic else None,
            out_of_cache=dict(big, traffic=(ub_traffic or {}).get("16384x8192")),
            loop_batch_on_4096_rows=K3, variants=variants)
    if args.full_solves:
        # the whole drop-in call, as main.cu -t times it: build + both phases + solution (problem
        # synthesised on the GPU and copied to the host first, outside the clock)
        # (at N GPUs: the whole solve on N row-block shards -- every rank calls twoPhaseMethod with
        # the whole problem and builds its own rows)
        out["full_solve"] = []
        for name in [c for c in args.full_solves.split(",") if c]:
            fn, fm, fseed = CONFIGS[name]
            prob = sx.generateRandomProblemDevice(fn, fm, fseed, 1, 100)
            torch.cuda.synchronize()
            barrier()
            t0 = time.perf_counter()
            res = sx.twoPhaseMethodEx(prob)
            dt = time.perf_counter() - t0
            prob.close()
            ph = (ctypes.c_double * 2)()
            sx.load().simplex_last_phase_seconds(ph)
            full = {"instance": name, "n": fn, "m": fm, "seed": fseed, "seconds": dt,
                    "status": sx.STATUS_NAMES.get(res.status, res.status), "pivots": list(res.pivots),
                    "objective": res.optimal_value,
                    "note": "twoPhaseMethod wall time incl. tableau build from host arrays, both phases and the solution",
                    "pivot_loop_s": [ph[0], ph[1]],
                    "pivots_per_s": [res.pivots[k] / ph[k] if ph[k] > 0 else None for k in (0, 1)],
                    "parity": solve_parity(name, res)}
            if name in REF_SOLVE:
                full["reference_pivots_per_s"] = [8981 / 68.33, 255 / 0.94]  # RTX 2070S, BASELINE.md §1
                full["reference_pivot_loop_s"] = REF_SOLVE[name]["pivot_loop_s"]
                full["reference_pivots"] = REF_SOLVE[name]["pivots"]
                full["pivots_match_reference"] = list(res.pivots) == REF_SOLVE[name]["pivots"]
            out["full_solve"].append(full)
    if rank == 0 and n_gpus == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(n, m, seed, CPU_SAMPLE[args.config], sx)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        sxdist.finalize()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
