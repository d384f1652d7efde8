"""Batched solve of B start/goal instances on the GPU (nlot_solve_batch, include/nlot.h).

`solve_batch` is the batched counterpart of `RunBenchmark.run()` (core/runner.py:44-153): same NLP,
same IPOPT-style algorithm, one instance per start/goal pair, all on the device.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np
import torch

from . import _abi
from ._lib import check, lib, require_gpu, stream_ptr
from .ops import DeviceMlp
from .problem import Problem


def _ptr(t: Optional[torch.Tensor]):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def solve_batch(problem: Problem, x0, xg, mlp: Optional[DeviceMlp] = None, options=None, X_init=None,
                device="cuda", workspace: Optional[torch.Tensor] = None):
    """Solve B instances.  x0, xg: [B, nx] (array or tensor).  Returns a dict of device tensors:
    X [B,N+1,nx], U [B,N,nu], S [B,N+1], cost [B], status [B] (0 solved, 1 max_iter,
    2 line-search failure, 3 numeric), iters [B]."""
    require_gpu()
    pc = problem.to_c()
    opt = options or _abi.gpu_options()
    x0 = torch.as_tensor(x0, dtype=torch.float64, device=device).contiguous()
    xg = torch.as_tensor(xg, dtype=torch.float64, device=device).contiguous()
    B, nx = x0.shape
    if nx != problem.nx or xg.shape != x0.shape:
        raise ValueError(f"x0/xg must be [B, {problem.nx}]")
    N, nu = problem.N, problem.nu
    if mlp is not None and not isinstance(mlp, DeviceMlp):
        mlp = mlp.device_mlp  # an L4CasADi / NNObstacle (nlotrajectories_amd.l4casadi)
    if problem.sdf == "mlp" and mlp is None:
        raise ValueError("learned-SDF problem needs a DeviceMlp, L4CasADi or NNObstacle")
    Xi = None
    if X_init is not None:
        Xi = torch.as_tensor(X_init, dtype=torch.float64, device=device).contiguous()
        assert Xi.shape == (B, N + 1, nx)
    f64 = dict(dtype=torch.float64, device=device)
    X = torch.empty(B, N + 1, nx, **f64)
    U = torch.empty(B, N, nu, **f64)
    S = torch.empty(B, N + 1, **f64)
    cost = torch.empty(B, **f64)
    status = torch.empty(B, dtype=torch.int32, device=device)
    iters = torch.empty(B, dtype=torch.int32, device=device)
    nbytes = lib().nlot_solve_workspace_size_slots(C.byref(pc), B, int(opt.max_active))
    if workspace is None or workspace.numel() < nbytes:
        workspace = torch.empty(nbytes, dtype=torch.uint8, device=device)
    check(lib().nlot_solve_batch(C.byref(pc), C.byref(opt), mlp.handle if mlp is not None else None, _ptr(x0),
                                 _ptr(xg), _ptr(Xi), _ptr(X), _ptr(U), _ptr(S), _ptr(cost), _ptr(status),
                                 _ptr(iters), B, _ptr(workspace), nbytes, stream_ptr()), "nlot_solve_batch")
    return dict(X=X, U=U, S=S, cost=cost, status=status, iters=iters)


def workspace_bytes(problem: Problem, B: int, slots: int = 0) -> int:
    """Workspace bytes for B instances through `slots` concurrent slots (0: all B at once)."""
    return int(lib().nlot_solve_workspace_size_slots(C.byref(problem.to_c()), B, slots))


def set_timing(every):
    """hipEvent timing inside nlot_solve_batch: False / 0 off, True / 1 every global step, k > 1 one step in k
    (NlotSolveStats.timed_* count the timed steps and their work; include/nlot.h)."""
    lib().nlot_set_timing(int(every))


def last_stats() -> dict:
    s = _abi.NlotSolveStats()
    lib().nlot_last_stats(C.byref(s))
    return {k: getattr(s, k) for k, _ in s._fields_}
