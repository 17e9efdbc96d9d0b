"""Loader of the HIP product library libsimplex_hip.so (ctypes, C-ABI of include/*.h).

torch (when installed) is imported BEFORE the library: torch ships its own HIP runtime and
RCCL with the same sonames (libamdhip64.so.7, librccl.so.1) as /opt/rocm.  Loading torch
first makes the library bind to those already-loaded copies, so one process holds one HIP
runtime.  There is no fallback: without the built library every entry point raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SIMPLEX_LIB_PATH") or os.path.join(_HERE, "libsimplex_hip.so")  # (diagnostic override)

c_double_p = ctypes.POINTER(ctypes.c_double)
c_int_p = ctypes.POINTER(ctypes.c_int)
c_ll_p = ctypes.POINTER(ctypes.c_longlong)


class ProblemT(ctypes.Structure):
    """problem_t (include/problem.h; reference problem.h:10-26)."""
    _fields_ = [
        ("constraintsMatrix", c_double_p),
        ("knownTermsVector", c_double_p),
        ("objectiveFunction", c_double_p),
        ("vars", ctypes.c_int),
        ("constraints", ctypes.c_int),
    ]


class TabularT(ctypes.Structure):
    """tabular_t (include/tabular.h; reference tabular.cuh:5-30)."""
    _fields_ = [
        ("problem", ctypes.POINTER(ProblemT)),
        ("table", c_double_p),
        ("knownTermsVector", c_double_p),
        ("constraintsMatrix", c_double_p),
        ("costsVector", c_double_p),
        ("pitch", ctypes.c_size_t),
        ("rows", ctypes.c_int),
        ("cols", ctypes.c_int),
    ]


class TimingT(ctypes.Structure):
    """simplex_timing_t (include/simplex_hip.h)."""
    _fields_ = [
        ("wall_ms", ctypes.c_double),
        ("update_ms", ctypes.c_double),
        ("pivots", ctypes.c_longlong),
        ("update_launches", ctypes.c_longlong),
        ("status", ctypes.c_int),
        ("width", ctypes.c_int),
        ("stored_width", ctypes.c_int),
        ("local_rows", ctypes.c_longlong),
        ("update_bytes", ctypes.c_double),
        ("swept_pivots", ctypes.c_longlong),
        ("swept_bytes", ctypes.c_double),
    ]


P_PROBLEM = ctypes.POINTER(ProblemT)
P_TABULAR = ctypes.POINTER(TabularT)

# name -> (restype, argtypes); every function declared in include/*.h
SIGNATURES = {
    # problem.h
    "readProblemFromFile": (P_PROBLEM, [ctypes.c_void_p]),
    "readRandomProblemFromFile": (P_PROBLEM, [ctypes.c_void_p]),
    "generateRandomProblem": (P_PROBLEM, [ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_int, ctypes.c_int]),
    "printProblemToStream": (None, [ctypes.c_void_p, P_PROBLEM]),
    "freeProblem": (None, [P_PROBLEM]),
    # tabular.h
    "newTabular": (P_TABULAR, [P_PROBLEM]),
    "printTableauToStream": (None, [ctypes.c_void_p, P_TABULAR, c_int_p]),
    "freeTabular": (None, [P_TABULAR]),
    # solver.h
    "solve": (ctypes.c_int, [P_TABULAR, c_int_p]),
    # twoPhaseMethod.h
    "twoPhaseMethod": (ctypes.c_int, [P_PROBLEM, c_double_p, c_double_p]),
    "enableBenchmarkMode": (None, []),
    "disableBenchmarkMode": (None, []),
    # simplex_hip.h
    "simplex_version": (ctypes.c_int, []),
    "simplex_set_verbose": (None, [ctypes.c_int]),
    "simplex_set_sweep_mfma": (None, [ctypes.c_int]),
    "simplex_set_batch": (None, [ctypes.c_int]),
    "simplex_set_device": (None, [ctypes.c_int]),
    "simplex_set_timer_dir": (None, [ctypes.c_char_p]),
    "simplex_dist_unique_id_size": (ctypes.c_int, []),
    "simplex_dist_get_unique_id": (ctypes.c_int, [ctypes.c_char_p]),
    "simplex_dist_init": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
    "simplex_dist_finalize": (ctypes.c_int, []),
    "simplex_set_virtual_ranks": (None, [ctypes.c_int]),
    "simplex_set_gpus": (None, [c_int_p, ctypes.c_int]),
    "simplex_gpus": (ctypes.c_int, [c_int_p, ctypes.c_int]),
    "simplex_set_force_exchange": (None, [ctypes.c_int]),
    "simplex_set_exchange_mode": (None, [ctypes.c_int]),
    "simplex_set_alias": (None, [ctypes.c_int]),
    "simplex_set_compact": (None, [ctypes.c_int]),
    "simplex_set_deactivate": (None, [ctypes.c_int]),
    "simplex_set_fused": (None, [ctypes.c_int]),
    "simplex_last_phase_seconds": (None, [ctypes.POINTER(ctypes.c_double)]),
    "simplex_last_objective_row": (ctypes.c_longlong, [ctypes.POINTER(ctypes.c_double), ctypes.c_longlong]),
    "simplex_set_p2p": (None, [ctypes.c_int]),
    "simplex_p2p_ready": (ctypes.c_int, []),
    "simplex_multi_gpu_mode": (ctypes.c_int, []),
    "simplex_set_update_waves": (None, [ctypes.c_double]),
    "simplex_set_regions": (None, [ctypes.c_int]),
    "simplex_set_mr_single_launch": (None, [ctypes.c_int]),
    "simplex_hang_recoveries": (ctypes.c_longlong, []),
    "simplex_fused_batches": (ctypes.c_longlong, []),
    "simplex_set_check_pivot_rows": (None, [ctypes.c_int]),
    "simplex_pivot_row_mismatches": (ctypes.c_longlong, []),
    "simplex_set_hang_inject": (None, [ctypes.c_longlong]),
    "simplex_set_hang_inject_slot": (None, [ctypes.c_int]),
    "simplex_set_first_batch_id": (None, [ctypes.c_uint]),
    "simplex_set_fine_pivot_rows": (None, [ctypes.c_int]),
    "simplex_set_replicated_objective": (None, [ctypes.c_int]),
    "simplex_set_blocked": (None, [ctypes.c_int]),
    "twoPhaseMethodEx": (ctypes.c_int, [P_PROBLEM, c_double_p, c_double_p, c_int_p, c_ll_p, ctypes.c_longlong]),
    "simplex_problem_from_arrays": (P_PROBLEM, [ctypes.c_int, ctypes.c_int, c_double_p, c_double_p, c_double_p]),
    "simplex_generate_problem_ex": (P_PROBLEM, [ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_int,
                                                ctypes.c_int, ctypes.c_int]),
    "simplex_free_problem_struct": (None, [P_PROBLEM]),
    "simplex_generate_problem_device": (P_PROBLEM, [ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_int,
                                                    ctypes.c_int, ctypes.c_int]),
    "simplex_session_open_generated": (ctypes.c_void_p, [ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_int,
                                                         ctypes.c_int, ctypes.c_int]),
    "simplex_dev_build_phase1_generated": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_int,
                                                          ctypes.c_int, c_double_p, ctypes.c_longlong, c_double_p,
                                                          c_int_p]),
    "simplex_session_open": (ctypes.c_void_p, [P_PROBLEM]),
    "simplex_session_pivots": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int,
                                              ctypes.POINTER(TimingT)]),
    "simplex_session_objective": (ctypes.c_double, [ctypes.c_void_p]),
    "simplex_session_tableau": (ctypes.c_longlong, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                                    ctypes.c_longlong, ctypes.POINTER(ctypes.c_double),
                                                    ctypes.POINTER(ctypes.c_int)]),
    "simplex_session_active_slacks": (ctypes.c_longlong, [ctypes.c_void_p]),
    "simplex_session_total_pivots": (ctypes.c_longlong, [ctypes.c_void_p]),
    "simplex_session_batch": (ctypes.c_int, [ctypes.c_void_p]),
    "simplex_session_launch_log": (ctypes.c_longlong, [ctypes.c_void_p, c_ll_p, c_double_p, ctypes.c_longlong]),
    "simplex_session_close": (None, [ctypes.c_void_p]),
    "simplex_session_stamps": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_ulonglong)]),
    "simplex_session_block_stamps": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_ulonglong),
                                                    ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_longlong]),
    "simplex_ipc_handles_size": (ctypes.c_int, []),
    "simplex_ipc_session_open": (ctypes.c_void_p, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_double_p,
                                                   ctypes.c_longlong, c_double_p, c_int_p, ctypes.c_char_p]),
    "simplex_ipc_session_connect": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p]),
    "simplex_session_sync_d": (ctypes.c_int, [ctypes.c_void_p]),
    "simplex_session_rows": (ctypes.c_longlong, [ctypes.c_void_p, c_double_p, ctypes.c_longlong, c_double_p,
                                                 c_int_p]),
    "simplex_bench_sweep": (ctypes.c_double, [ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_int, ctypes.c_int, c_double_p]),
    "simplex_dev_argmin": (ctypes.c_longlong, [c_double_p, ctypes.c_longlong, c_double_p]),
    "simplex_dev_pivots": (ctypes.c_int, [c_double_p, ctypes.c_longlong, ctypes.c_longlong, ctypes.c_longlong,
                                          c_double_p, c_int_p, ctypes.c_longlong, c_ll_p]),
    "simplex_dev_update_objective": (ctypes.c_int, [c_double_p, ctypes.c_longlong, ctypes.c_longlong,
                                                    ctypes.c_longlong, c_int_p, c_double_p]),
    "simplex_dev_build_phase1": (ctypes.c_int, [P_PROBLEM, c_double_p, ctypes.c_longlong, c_double_p, c_int_p]),
}

_lib = None


def load():
    """Return the loaded library (raises if the HIP extension was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"simplexoncuda_amd: HIP library {LIB_PATH} is missing; run "
            "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
    try:
        import torch  # noqa: F401  -- share torch's HIP runtime / RCCL (see module docstring)
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib
