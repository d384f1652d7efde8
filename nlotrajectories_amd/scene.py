"""Host-side scene SDFs for reporting (the CLI's SDF-quality metrics), not the solve path.

Exact and smoothed ("approximated") signed distances of the analytic obstacles, vectorised over numpy
grids, following the reference's obstacle classes: circle (core/sdf/casadi.py:33-41, its approximated
SDF is the exact one), square (exact box distance :58-72, smooth soft-abs/soft-max/soft-min version
:74-118 with eps 1e-6) and their union (exact: min; approximated: soft-min with alpha 10,
core/utils.py:18-33, :385-386).  The GPU solver evaluates the same smoothed SDF on the device
(csrc/nlot_device.h).
"""
from __future__ import annotations

import numpy as np

_E = 1e-6


def _circle(o, x, y):
    return np.sqrt((x - o["center"][0]) ** 2 + (y - o["center"][1]) ** 2) - (o["radius"] + o.get("margin", 0.0))


def _square_exact(o, x, y):
    h = o["size"] / 2 + o.get("margin", 0.0)
    dx = np.abs(x - o["center"][0]) - h
    dy = np.abs(y - o["center"][1]) - h
    return np.hypot(np.maximum(dx, 0), np.maximum(dy, 0)) + np.minimum(np.maximum(dx, dy), 0)


def _smax(a, b):
    return 0.5 * (a + b + np.sqrt((a - b) ** 2 + _E))


def _smin(a, b):
    return 0.5 * (a + b - np.sqrt((a - b) ** 2 + _E))


def _square_smooth(o, x, y):
    h = o["size"] / 2 + o.get("margin", 0.0)
    ax_ = np.sqrt((x - o["center"][0]) ** 2 + _E) - h
    ay_ = np.sqrt((y - o["center"][1]) ** 2 + _E) - h
    outside = np.sqrt(_smax(ax_, 0.0) ** 2 + _smax(ay_, 0.0) ** 2)
    return outside + _smin(_smax(ax_, ay_), 0.0)


def soft_min(values, alpha: float = 10.0):
    """-(1/alpha) log sum exp(-alpha v), stabilised by the minimum."""
    v = np.stack(values, 0)
    m = v.min(0)
    return m - np.log(np.exp(-alpha * (v - m)).sum(0)) / alpha


def exact_sdf(obstacles, x, y):
    vals = []
    for o in obstacles:
        if o["type"] == "circle":
            vals.append(_circle(o, x, y))
        elif o["type"] == "square":
            vals.append(_square_exact(o, x, y))
        else:
            raise NotImplementedError(f"exact SDF of {o['type']!r} obstacles (DESIGN.md §9)")
    return np.min(np.stack(vals, 0), 0)


def approximated_sdf(obstacles, x, y, alpha: float = 10.0):
    vals = []
    for o in obstacles:
        if o["type"] == "circle":
            vals.append(_circle(o, x, y))
        elif o["type"] == "square":
            vals.append(_square_smooth(o, x, y))
        else:
            raise NotImplementedError(f"smoothed SDF of {o['type']!r} obstacles (DESIGN.md §9)")
    return soft_min(vals, alpha)


# SDF-quality metrics of an approximated SDF against the exact one on a grid (the reference's
# core/metrics.py definitions: MSE, IoU of the sdf < 0 sets, and the Hausdorff / Chamfer distances and
# surface loss of the |sdf| < eps level sets)
def mse(target, pred):
    return float(np.mean((target - pred) ** 2))


def iou(target, pred, threshold=0.0):
    a, b = target < threshold, pred < threshold
    union = np.logical_or(a, b).sum()
    inter = np.logical_and(a, b).sum()
    return 1.0 if union == 0 and inter == 0 else (0.0 if union == 0 else float(inter / union))


def _surface(sdf, X, Y, eps):
    pts = np.stack([X, Y], -1).reshape(-1, 2)
    return pts[np.abs(sdf.ravel()) < eps]


def _nearest(a, b, chunk=2048):
    out = np.empty(len(a))
    for i in range(0, len(a), chunk):
        out[i:i + chunk] = np.sqrt(((a[i:i + chunk, None, :] - b[None]) ** 2).sum(-1)).min(1)
    return out


def hausdorff(target, pred, X, Y, eps=1e-2):
    p, t = _surface(pred, X, Y, eps), _surface(target, X, Y, eps)
    if len(p) == 0 or len(t) == 0:
        return None
    return float(max(_nearest(p, t).max(), _nearest(t, p).max()))


def chamfer(target, pred, X, Y, eps=1e-2):
    p, t = _surface(pred, X, Y, eps), _surface(target, X, Y, eps)
    if len(p) == 0 or len(t) == 0:
        return None
    return float((_nearest(p, t).mean() + _nearest(t, p).mean()) / 2)


def surface_loss(target, pred, eps=1e-2):
    m = np.abs(target.ravel()) < eps
    return float(np.mean(pred.ravel()[m] ** 2)) if m.any() else None
