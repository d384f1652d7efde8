"""Seeded synthetic start/goal batches (SURVEY.md §8d 'Synthetic inputs')."""
from __future__ import annotations

import math

import numpy as np

from .problem import Problem


def _corners(problem: Problem, x, y, th):
    c, s = np.cos(th), np.sin(th)
    pts = [(x + c * bx - s * by, y + s * bx + c * by) for bx, by in problem.body]
    return np.stack([np.stack(p, -1) for p in pts], -2)  # [..., n_body, 2]


def sample_start_goal(problem: Problem, B: int, seed: int = 0, sdf=None, lo=(-0.3, -0.3), hi=(1.3, 1.3),
                      min_clear: float = 0.02, min_dist: float = 0.3, rank: int = 0):
    """B start/goal pairs for `problem` (unicycle-style state: x, y, theta, 0...).

    Positions are uniform in the box [lo, hi]^2 ([-0.3, 1.3]^2); the heading of
    start and goal is the straight-line direction; the remaining states are 0.  A pair is rejected
    unless every footprint corner at start and goal has sdf >= min_clear and the two positions are
    at least `min_dist` apart.  `sdf(points[P,2]) -> values[P]` is the scene SDF used for rejection.
    The generator is numpy's PCG64 seeded with seed + 1000003 * rank (disjoint per rank).
    """
    rng = np.random.default_rng(seed + 1000003 * rank)
    nx = problem.nx
    out0, outg = [], []
    lo, hi = np.asarray(lo, float), np.asarray(hi, float)
    rounds = 0
    while sum(len(a) for a in out0) < B:
        rounds += 1
        if rounds > 64 and sum(len(a) for a in out0) < rounds:
            raise RuntimeError("sample_start_goal: the scene leaves almost no free start/goal pairs in the box")
        n = max(4 * B, 1024)
        s = lo + (hi - lo) * rng.random((n, 2))
        g = lo + (hi - lo) * rng.random((n, 2))
        ok = np.linalg.norm(g - s, axis=1) >= min_dist
        th = np.arctan2(g[:, 1] - s[:, 1], g[:, 0] - s[:, 0])
        if sdf is not None:
            cs = _corners(problem, s[:, 0], s[:, 1], th) if problem.shape != "dot" else s[:, None, :]
            cg = _corners(problem, g[:, 0], g[:, 1], th) if problem.shape != "dot" else g[:, None, :]
            vs = np.asarray(sdf(cs.reshape(-1, 2))).reshape(n, -1).min(1)
            vg = np.asarray(sdf(cg.reshape(-1, 2))).reshape(n, -1).min(1)
            ok &= (vs >= min_clear) & (vg >= min_clear)
        x0 = np.zeros((n, nx))
        xg = np.zeros((n, nx))
        x0[:, :2], xg[:, :2] = s, g
        if nx >= 3 and problem.dynamics not in ("point_1st", "point_2nd"):
            x0[:, 2] = th
            xg[:, 2] = th
        out0.append(x0[ok])
        outg.append(xg[ok])
    return np.concatenate(out0)[:B], np.concatenate(outg)[:B]
