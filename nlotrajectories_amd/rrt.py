"""RRT initial guesses on the GPU: the reference's RRTInitializer (core/trajectory_initialization.py:58-239)
batched over instances (nlot_rrt_init, csrc/nlot_rrt.hip).

`RRTInitializer` keeps the reference's constructor arguments (N = number of points, x0, x_goal, dt, sdf_func,
geometry, bounds, step_size, max_iter, margin, goal_sample_rate) where they make sense for a batched call:
the scene comes from the `Problem` (its analytic obstacles, whose exact SDF the reference passes as
`sdf_func=obstacles.sdf`), the footprint from `Problem.shape`.  Randomness is a seeded counter-based stream
(the reference uses Python's unseeded global `random`)."""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _abi
from ._lib import check, lib, require_gpu, stream_ptr
from .problem import Problem

CHUNK = 4096  # instances per nlot_rrt_init call: the workspace is bounded by the chunk (4 GB for benchmark 6's
#               max_iter 5000, 16 GB for all 16,384 instances at once); the draws are keyed by the global instance
#               index (NlotRrtOptions.first_instance), so the result is the same as one call


def rrt_options(bounds, step_size=0.05, max_iter=1000, margin=0.01, goal_sample_rate=0.05, seed=0):
    o = _abi.NlotRrtOptions()
    (o.bounds[0][0], o.bounds[0][1]), (o.bounds[1][0], o.bounds[1][1]) = [tuple(map(float, r)) for r in bounds]
    o.step_size, o.margin, o.goal_sample_rate = float(step_size), float(margin), float(goal_sample_rate)
    o.seed, o.max_iter = int(seed) & (2 ** 64 - 1), int(max_iter)
    return o


def rrt_initial_guess(problem: Problem, x0, xg, bounds, step_size=0.05, max_iter=1000, margin=0.01,
                      goal_sample_rate=0.05, seed=0, device="cuda"):
    """Batched RRTInitializer.get_initial_guess: (X_init [B, N+1, nx] fp64 device, ok [B] bool device).  ok is
    False where the reference raises RuntimeError("RRT failed to find a path within max_iter."); that
    instance's X_init is the straight line."""
    require_gpu()
    if not problem.obstacles:
        raise ValueError("the RRT plans against the scene's exact SDF: the problem needs its analytic obstacles")
    pc = problem.with_(sdf="analytic").to_c()
    o = rrt_options(bounds, step_size, max_iter, margin, goal_sample_rate, seed)
    x0 = torch.as_tensor(x0, dtype=torch.float64, device=device).contiguous()
    xg = torch.as_tensor(xg, dtype=torch.float64, device=device).contiguous()
    B, nx = x0.shape
    if nx != problem.nx or xg.shape != x0.shape:
        raise ValueError(f"x0/xg must be [B, {problem.nx}]")
    X = torch.empty(B, problem.N + 1, nx, dtype=torch.float64, device=device)
    ok = torch.empty(B, dtype=torch.int32, device=device)
    nbytes = lib().nlot_rrt_workspace_size(C.byref(o), min(B, CHUNK))
    # per call, on the caller's stream: two calls on different streams or threads never share a workspace (torch's
    # caching allocator reuses the memory; 25 (max_iter + 2) doubles per instance of one chunk)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=device)
    for c0 in range(0, B, CHUNK):
        n = min(CHUNK, B - c0)
        o.first_instance = c0
        check(lib().nlot_rrt_init(C.byref(pc), C.byref(o), x0[c0].data_ptr(), xg[c0].data_ptr(), X[c0].data_ptr(),
                                  ok[c0:].data_ptr(), n, ws.data_ptr(), nbytes, stream_ptr()), "nlot_rrt_init")
    return X, ok.bool()


class RRTInitializer:
    """trajectory_initialization.py:58-239 with the reference's argument names; `problem` carries the scene and
    the footprint (sdf_func / geometry of the reference)."""

    def __init__(self, N, x0, x_goal, dt, problem: Problem, bounds, step_size=0.05, max_iter=1000, margin=0.01,
                 goal_sample_rate=0.05, seed=0):
        if N != problem.N + 1:
            raise ValueError("N is the number of points of the returned trajectory (solver N + 1)")
        self.N, self.x0, self.x_goal, self.dt, self.problem = N, np.asarray(x0, float), np.asarray(x_goal, float), dt, problem
        self.kw = dict(bounds=bounds, step_size=step_size, max_iter=max_iter, margin=margin,
                       goal_sample_rate=goal_sample_rate, seed=seed)

    def get_initial_guess(self) -> np.ndarray:
        X, ok = rrt_initial_guess(self.problem, self.x0[None], self.x_goal[None], **self.kw)
        if not bool(ok[0]):
            raise RuntimeError("RRT failed to find a path within max_iter.")
        return X[0].cpu().numpy()
