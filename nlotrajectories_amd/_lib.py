"""Loader for libnlot.so (the HIP kernels behind the C ABI of include/nlot.h).

There is no CPU fallback: every compute entry point of this package goes through this library, and
importing a compute function without the built library or without a GPU raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

from . import _abi

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# NLOT_LIB selects an alternative in-tree build (e.g. the phase-timer build libnlot_prof.so)
LIB_PATH = os.path.join(PKG_DIR, os.environ.get("NLOT_LIB", "libnlot.so"))
CSRC = os.path.join(PKG_DIR, "csrc")

# symbols include/nlot.h declares (checked by tests/test_abi.py)
EXPORTED = [
    "nlot_abi_version", "nlot_last_error", "nlot_default_options", "nlot_mlp_create", "nlot_mlp_create_ex", "nlot_mlp_destroy",
    "nlot_sdf_mlp_eval", "nlot_solve_workspace_size", "nlot_solve_workspace_size_slots", "nlot_solve_batch", "nlot_set_timing",
    "nlot_last_stats", "nlot_casadi_bind", "nn_sdf_n_in", "nn_sdf_n_out", "nn_sdf_sparsity_in",
    "nn_sdf_sparsity_out", "nn_sdf", "jac_nn_sdf_n_in", "jac_nn_sdf_n_out", "jac_nn_sdf",
    "adj1_nn_sdf_n_in", "adj1_nn_sdf_n_out", "adj1_nn_sdf", "jac_adj1_nn_sdf_n_in",
    "jac_adj1_nn_sdf_n_out", "jac_adj1_nn_sdf", "nlot_rrt_workspace_size", "nlot_rrt_init",
]


class NlotError(RuntimeError):
    pass


def build(force: bool = False) -> str:
    """Compile libnlot.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    args = ["make", "-C", CSRC, "-j8"]
    if force:
        subprocess.run(["make", "-C", CSRC, "clean"], check=True, capture_output=True)
    subprocess.run(args, check=True)
    return LIB_PATH


_lib = None


def lib():
    """The loaded library with argtypes set.  Raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NlotError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'` "
                        "(no CPU fallback exists)")
    L = C.CDLL(LIB_PATH)
    vp, dp, fp, i32p = C.c_void_p, C.POINTER(C.c_double), C.c_void_p, C.c_void_p
    L.nlot_abi_version.restype = C.c_int32
    L.nlot_last_error.restype = C.c_char_p
    L.nlot_default_options.argtypes = [C.POINTER(_abi.NlotSolverOptions)]
    L.nlot_mlp_create.argtypes = [C.POINTER(_abi.NlotMlpDesc)]
    L.nlot_mlp_create.restype = vp
    L.nlot_mlp_create_ex.argtypes = [C.POINTER(_abi.NlotMlpDesc), C.c_int32]
    L.nlot_mlp_create_ex.restype = vp
    L.nlot_mlp_destroy.argtypes = [vp]
    L.nlot_sdf_mlp_eval.argtypes = [vp, vp, C.c_int64, vp, vp, vp, vp, vp]
    L.nlot_sdf_mlp_eval.restype = C.c_int32
    L.nlot_solve_workspace_size.argtypes = [C.POINTER(_abi.NlotProblem), C.c_int64]
    L.nlot_solve_workspace_size.restype = C.c_size_t
    L.nlot_solve_workspace_size_slots.argtypes = [C.POINTER(_abi.NlotProblem), C.c_int64, C.c_int32]
    L.nlot_solve_workspace_size_slots.restype = C.c_size_t
    L.nlot_solve_batch.argtypes = [C.POINTER(_abi.NlotProblem), C.POINTER(_abi.NlotSolverOptions), vp, vp, vp, vp,
                                   vp, vp, vp, vp, vp, vp, C.c_int64, vp, C.c_size_t, vp]
    L.nlot_solve_batch.restype = C.c_int32
    L.nlot_set_timing.argtypes = [C.c_int32]
    L.nlot_last_stats.argtypes = [C.POINTER(_abi.NlotSolveStats)]
    L.nlot_rrt_workspace_size.argtypes = [C.POINTER(_abi.NlotRrtOptions), C.c_int64]
    L.nlot_rrt_workspace_size.restype = C.c_size_t
    L.nlot_rrt_init.argtypes = [C.POINTER(_abi.NlotProblem), C.POINTER(_abi.NlotRrtOptions), vp, vp, vp, vp, C.c_int64,
                                vp, C.c_size_t, vp]
    L.nlot_rrt_init.restype = C.c_int32
    L.nlot_casadi_bind.argtypes = [vp]
    L.nlot_casadi_bind.restype = C.c_int32
    if L.nlot_abi_version() != 15:
        raise NlotError("libnlot.so ABI version mismatch")
    _lib = L
    return L


def check(rc: int, what: str):
    if rc != 0:
        raise NlotError(f"{what} failed ({rc}): {lib().nlot_last_error().decode()}")


def require_gpu():
    import torch

    if not torch.cuda.is_available():
        raise NlotError("nlotrajectories_amd needs a ROCm GPU (MI355X); no CPU fallback exists")


def stream_ptr(stream=None):
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)
