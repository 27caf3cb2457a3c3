"""ctypes binding of ``libcarmpc.so`` -- the C ABI declared in ``include/carmpc.h``.

The library is built in-tree (``python -m carmpc_amd.build`` or
``__graft_entry__.build()``).  If the library is missing every entry point raises
``CarMPCNativeError``; the device entry points need a GPU, the ``carmpc_cpu_*`` twins
(the host's CPU QP path, as in the reference) do not.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# CARMPC_LIB selects another in-tree build of the same ABI (e.g. the phase-timing
# profiling build of tools/phase_timing.py); default: the production library.
LIB_PATH = os.environ.get("CARMPC_LIB") or os.path.join(_HERE, "libcarmpc.so")

# status codes (carmpc.h)
OPTIMAL, PRIMAL_INFEASIBLE, MAX_ITER, NUMERICAL = 0, 1, 2, 3
STATUS_NAMES = {OPTIMAL: "optimal", PRIMAL_INFEASIBLE: "primal_infeasible", MAX_ITER: "max_iter",
                NUMERICAL: "numerical"}

# symbols declared in include/carmpc.h (checked by tests/test_abi.py)
EXPORTS = ("carmpc_problem_create", "carmpc_problem_create_dense", "carmpc_problem_destroy",
           "carmpc_problem_info", "carmpc_problem_get", "carmpc_solve_batch", "carmpc_solve_segments",
           "carmpc_observer_batch", "carmpc_plant_step_batch", "carmpc_canonical_flops_per_iter",
           "carmpc_last_error", "carmpc_version", "carmpc_problem_kernel",
           "carmpc_executed_flops_per_iter", "carmpc_issued_flops_per_iter", "carmpc_problem_set_disturbance", "carmpc_solve_batch_dist",
           "carmpc_observer_dist_batch", "carmpc_closed_loop_batch", "carmpc_lp_batch",
           "carmpc_hetero_create", "carmpc_hetero_destroy", "carmpc_hetero_linearize", "carmpc_hetero_solve",
           "carmpc_hetero_get", "carmpc_solve_batch_noalloc",
           "carmpc_problem_set_observer", "carmpc_cpu_problem_create", "carmpc_cpu_problem_destroy",
           "carmpc_cpu_problem_info", "carmpc_cpu_problem_set_disturbance", "carmpc_cpu_solve_batch",
           "carmpc_cpu_solve_batch_dist")

# outcomes of carmpc_closed_loop_batch (carmpc.h)
LOOP_RUNNING, LOOP_REACHED, LOOP_INFEASIBLE, LOOP_INPUT_VIOLATION, LOOP_TIMEOUT, LOOP_SOLVER_FAILURE = -1, 0, 1, 2, 3, 4
LOOP_NAMES = {LOOP_RUNNING: "running", LOOP_REACHED: "reached", LOOP_INFEASIBLE: "infeasible",
              LOOP_INPUT_VIOLATION: "input_violation", LOOP_TIMEOUT: "timeout", LOOP_SOLVER_FAILURE: "solver_failure"}


class CarMPCNativeError(RuntimeError):
    """Raised when the HIP library is missing or a C-ABI call fails."""


class ModelDesc(ctypes.Structure):
    """carmpc_model_desc (include/carmpc.h)."""
    _dp = ctypes.POINTER(ctypes.c_double)
    _fields_ = [("N", ctypes.c_int32), ("nx", ctypes.c_int32), ("nu", ctypes.c_int32),
                ("A", _dp), ("B", _dp), ("Q", _dp), ("R", _dp), ("P", _dp),
                ("n_state_rows", ctypes.c_int32), ("state_A", _dp), ("state_b", _dp),
                ("n_term_rows", ctypes.c_int32), ("term_A", _dp), ("term_b", _dp),
                ("u_lower", _dp), ("u_upper", _dp), ("goal", _dp)]


class LoopDesc(ctypes.Structure):
    """carmpc_loop_desc (include/carmpc.h)."""
    _dp = ctypes.POINTER(ctypes.c_double)
    _fields_ = [("mode", ctypes.c_int32), ("steps_update", ctypes.c_int32), ("last_step", ctypes.c_int32),
                ("ny", ctypes.c_int32), ("dt", ctypes.c_double), ("l1", ctypes.c_double),
                ("goal_tol", ctypes.c_double), ("goal", _dp), ("C", _dp), ("L", _dp), ("Cd", _dp), ("L2", _dp),
                ("Bd", _dp)]


class HeteroDesc(ctypes.Structure):
    """carmpc_hetero_desc (include/carmpc.h)."""
    _dp = ctypes.POINTER(ctypes.c_double)
    _fields_ = [("N", ctypes.c_int32), ("dt", ctypes.c_double), ("l1", ctypes.c_double), ("Q", _dp), ("R", _dp),
                ("n_state_rows", ctypes.c_int32), ("state_A", _dp), ("state_b", _dp),
                ("n_term_rows", ctypes.c_int32), ("term_A", _dp), ("term_b", _dp),
                ("u_lower", _dp), ("u_upper", _dp), ("goal", _dp)]


class Settings(ctypes.Structure):
    """carmpc_settings (include/carmpc.h)."""
    _fields_ = [("tol", ctypes.c_double), ("tol_mu", ctypes.c_double), ("max_iter", ctypes.c_int32),
                ("kernel", ctypes.c_int32)]


_lib = None


def load():
    """Load libcarmpc.so (once).  Raises CarMPCNativeError if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise CarMPCNativeError(f"{LIB_PATH} not found: build it with `python -m carmpc_amd.build` "
                                "(hipcc --offload-arch=gfx950); the GPU kernels and the host path "
                                "(carmpc_cpu_*) both live in that library, nothing runs without it")
    lib = ctypes.CDLL(LIB_PATH)
    vp, dp, ip = ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int32)
    i32, i64 = ctypes.c_int32, ctypes.c_int64
    sig = {
        "carmpc_problem_create": ([ctypes.POINTER(ModelDesc), ctypes.POINTER(vp)], ctypes.c_int),
        "carmpc_problem_create_dense": ([i32, i32, i32, dp, dp, dp, dp, dp, dp, dp, dp, ctypes.POINTER(vp)],
                                        ctypes.c_int),
        "carmpc_problem_destroy": ([vp], None),
        "carmpc_problem_info": ([vp, ip, ip, ip, ip, ip], ctypes.c_int),
        "carmpc_problem_get": ([vp, dp, dp, dp, dp, dp, dp, dp, ip], ctypes.c_int),
        "carmpc_solve_batch": ([vp, i64, vp, vp, vp, vp, vp, ctypes.POINTER(Settings), vp], ctypes.c_int),
        "carmpc_solve_batch_noalloc": ([vp, i64, vp, vp, vp, vp, vp, ctypes.POINTER(Settings), vp], ctypes.c_int),
        "carmpc_problem_set_observer": ([vp, i32, dp, dp, dp, dp, dp], ctypes.c_int),
        "carmpc_cpu_problem_create": ([ctypes.POINTER(ModelDesc), ctypes.POINTER(vp)], ctypes.c_int),
        "carmpc_cpu_problem_destroy": ([vp], None),
        "carmpc_cpu_problem_info": ([vp, ip, ip, ip, ip, ip], ctypes.c_int),
        "carmpc_cpu_problem_set_disturbance": ([vp, dp], ctypes.c_int),
        "carmpc_cpu_solve_batch": ([vp, i64, dp, dp, dp, ip, ip, ctypes.POINTER(Settings), i32], ctypes.c_int),
        "carmpc_cpu_solve_batch_dist": ([vp, i64, dp, dp, dp, dp, ip, ip, ctypes.POINTER(Settings), i32],
                                        ctypes.c_int),
        "carmpc_solve_segments": ([ctypes.POINTER(vp), i32, ctypes.POINTER(i64), vp, vp, vp, i64, vp, vp,
                                   ctypes.POINTER(Settings), vp], ctypes.c_int),
        "carmpc_observer_batch": ([vp, i64, vp, i32, dp, dp, vp, vp, i64, vp], ctypes.c_int),
        "carmpc_plant_step_batch": ([i64, vp, vp, i64, ctypes.c_double, ctypes.c_double, vp, vp], ctypes.c_int),
        "carmpc_canonical_flops_per_iter": ([i32, i32], ctypes.c_double),
        "carmpc_last_error": ([], ctypes.c_char_p),
        "carmpc_version": ([], ctypes.c_char_p),
        "carmpc_problem_kernel": ([vp], ctypes.c_int),
        "carmpc_executed_flops_per_iter": ([vp, i32], ctypes.c_double),
        "carmpc_issued_flops_per_iter": ([vp, i32], ctypes.c_double),
        "carmpc_problem_set_disturbance": ([vp, dp], ctypes.c_int),
        "carmpc_solve_batch_dist": ([vp, i64, vp, vp, vp, vp, vp, vp, ctypes.POINTER(Settings), vp], ctypes.c_int),
        "carmpc_observer_dist_batch": ([vp, i64, vp, i32, dp, dp, dp, dp, dp, vp, vp, vp, i64, vp], ctypes.c_int),
        "carmpc_lp_batch": ([i64, i32, vp, vp, vp, vp, vp, vp, vp, ctypes.c_double, vp, vp, vp, vp, vp],
                            ctypes.c_int),
        "carmpc_hetero_create": ([ctypes.POINTER(HeteroDesc), i64, ctypes.POINTER(vp)], ctypes.c_int),
        "carmpc_hetero_destroy": ([vp], None),
        "carmpc_hetero_linearize": ([vp, vp, vp, vp], ctypes.c_int),
        "carmpc_hetero_solve": ([vp, vp, vp, vp, vp, vp, ctypes.POINTER(Settings), vp], ctypes.c_int),
        "carmpc_hetero_get": ([vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp], ctypes.c_int),
        "carmpc_closed_loop_batch": ([vp, i64, ctypes.POINTER(LoopDesc), vp, vp, vp, vp, vp, vp, vp, i32,
                                      ctypes.POINTER(Settings), vp], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().carmpc_last_error().decode(errors="replace")
        raise CarMPCNativeError(f"{what} failed ({rc}): {msg}")


def version() -> str:
    return load().carmpc_version().decode()
