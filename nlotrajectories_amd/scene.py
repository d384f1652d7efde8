"""Host-side scene SDFs for reporting (the CLI's SDF-quality metrics), not the solve path.

Exact and smoothed ("approximated") signed distances of the analytic obstacles, vectorised over numpy
grids, following the reference's obstacle classes: circle (core/sdf/casadi.py:33-41, its approximated
SDF is the exact one), square (exact box distance :58-72, smooth soft-abs/soft-max/soft-min version
:74-118 with eps 1e-6), polygon (exact: distance to the boundary signed by containment, :135-148, as
shapely computes it; approximated :150-186), elliptical ring (a polygon), trapezoid (exact: the polygon's;
approximated :317-374), convex elliptic ring / discr_s (MultiObstacles of trapezoids: exact min, approximated
soft_min) and their union (exact: min; approximated: soft-min with alpha 10, core/utils.py:18-33,
:385-386).  The composite obstacles are expanded into primitives by obstacles.expand, as the solver's
NlotProblem carries them.  The GPU solver evaluates the same smoothed SDF on the device (csrc/nlot_device.h).
"""
from __future__ import annotations

import numpy as np

from . import _abi
from .obstacles import expand

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


def _poly_exact(V, x, y):
    """Signed distance to a simple polygon: distance to its boundary (the edge segments), negative inside
    (even-odd crossing test) — what PolygonObstacle.sdf computes with shapely (casadi.py:135-148)."""
    d = np.full(np.shape(x), np.inf)
    inside = np.zeros(np.shape(x), bool)
    n = len(V)
    for e in range(n):
        (x0, y0), (x1, y1) = V[e], V[(e + 1) % n]
        dx, dy = x1 - x0, y1 - y0
        t = np.clip(((x - x0) * dx + (y - y0) * dy) / (dx * dx + dy * dy), 0.0, 1.0)
        d = np.minimum(d, np.hypot(x - (x0 + t * dx), y - (y0 + t * dy)))
        crosses = (y0 > y) != (y1 > y)
        with np.errstate(divide="ignore", invalid="ignore"):
            xi = x0 + (y - y0) * dx / (y1 - y0)
        inside ^= crosses & (x < xi)
    return np.where(inside, -d, d)


def _poly_smooth(V, c, margin, x, y, alpha):
    """PolygonObstacle.approximated_sdf (casadi.py:150-186)."""
    dists = []
    n = len(V)
    for e in range(n):
        (x0, y0), (x1, y1) = V[e], V[(e + 1) % n]
        dx, dy = x1 - x0, y1 - y0
        t = np.minimum(1.0, np.maximum(0.0, ((x - x0) * dx + (y - y0) * dy) / (dx ** 2 + dy ** 2 + 1e-6)))
        dists.append(np.sqrt((x - (x0 + t * dx)) ** 2 + (y - (y0 + t * dy)) ** 2))
    return np.tanh(100 * ((x - c[0]) * (y - c[1]))) * _soft_min_ref(dists, alpha) - margin


def _trap_smooth(V, margin, x, y):
    """TrapezoidObstacle.approximated_sdf (casadi.py:317-374), soft helpers with eps 1e-8."""
    sabs = lambda v: np.sqrt(v ** 2 + 1e-8)  # noqa: E731
    smax = lambda a, b: 0.5 * (a + b + sabs(a - b))  # noqa: E731
    smin = lambda a, b: 0.5 * (a + b - sabs(a - b))  # noqa: E731
    n = len(V)
    hp, seg = [], []
    for e in range(n):
        (x0, y0), (x1, y1) = V[e], V[(e + 1) % n]
        ex, ey = x1 - x0, y1 - y0
        nl = np.sqrt(ey ** 2 + ex ** 2 + 1e-6)
        hp.append(((ey / nl) * (x - x0) + (-ex / nl) * (y - y0)) - margin)
        t = smin(1, smax(0, ((x - x0) * ex + (y - y0) * ey) / (ex ** 2 + ey ** 2 + 1e-6)))
        seg.append(np.sqrt((x - (x0 + t * ex)) ** 2 + (y - (y0 + t * ey)) ** 2 + 1e-6))
    inner, outside = hp[0], seg[0]
    for v in hp[1:]:
        inner = smax(inner, v)
    for v in seg[1:]:
        outside = smin(outside, v)
    return outside + smin(inner, 0) - margin


def _soft_min_ref(values, alpha):
    """soft_min exactly as core/utils.py:18-33 writes it (no shift)."""
    return -1.0 / alpha * np.log(np.sum(np.exp(-alpha * np.stack(values, 0)), axis=0))


def _terms(obstacles, x, y, prim_fn, combine):
    """Scene terms: one per top-level obstacle; a group's primitives combined by `combine` first."""
    prims, verts = expand(obstacles)
    out, grp, cur = [], [], None
    for q in prims:
        v = prim_fn(q, verts[q["v0"]:q["v0"] + q["nv"]], x, y)
        if q["group"] < 0:
            if grp:
                out.append(combine(grp))
                grp = []
            out.append(v)
        else:
            if grp and q["group"] != cur:
                out.append(combine(grp))
                grp = []
            cur = q["group"]
            grp.append(v)
    if grp:
        out.append(combine(grp))
    return out


def _prim(q, V, x, y, exact, alpha):
    o = {"center": (q["cx"], q["cy"]), "radius": q["size"], "size": q["size"], "margin": q["margin"]}
    if q["type"] == _abi.OBS_CIRCLE:
        return _circle(o, x, y)
    if q["type"] == _abi.OBS_SQUARE:
        return _square_exact(o, x, y) if exact else _square_smooth(o, x, y)
    if exact:  # PolygonObstacle.sdf: distance to the boundary signed by containment, minus the margin
        return _poly_exact(V, x, y) - q["margin"]
    if q["type"] == _abi.OBS_POLYGON:
        return _poly_smooth(V, (q["cx"], q["cy"]), q["margin"], x, y, alpha)
    return _trap_smooth(V, q["margin"], x, y)


def exact_sdf(obstacles, x, y):
    vals = _terms(obstacles, x, y, lambda q, V, x, y: _prim(q, V, x, y, True, 10.0),
                  lambda g: np.min(np.stack(g, 0), 0))
    return np.min(np.stack(vals, 0), 0)


def approximated_sdf(obstacles, x, y, alpha: float = 10.0):
    vals = _terms(obstacles, x, y, lambda q, V, x, y: _prim(q, V, x, y, False, alpha),
                  lambda g: _soft_min_ref(g, alpha))
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
