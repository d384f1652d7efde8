"""TEST INFRASTRUCTURE ONLY (never imported by the product): a CPU restatement of the reference's RRTInitializer
(core/trajectory_initialization.py:58-239) that checks the GPU's nlot_rrt_init (csrc/nlot_rrt.hip).

It follows the reference line by line — tree growth with goal bias and step-size steering, nearest node by
np.argmin, point-inflation collision checks against the scene's exact SDF (MultiObstacle.sdf,
casadi.py:381-383), insert_intermediate_points, _shortcut_path, scipy's CubicSpline (the reference's own
dependency) resampled to N points, lift with zeros — with two substitutions, both shared with the GPU:
* draws: a counter-based splitmix64 stream of (seed, instance, iteration, draw) instead of Python's global
  `random` (which the reference never seeds);
* exact polygon SDF: the boundary distance signed by an even-odd containment test, in place of shapely
  (absent here).
"""
from __future__ import annotations

import math
import sys
import os

import numpy as np
from scipy.interpolate import CubicSpline

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nlotrajectories_amd import _abi  # noqa: E402
from nlotrajectories_amd.obstacles import expand  # noqa: E402

M64 = (1 << 64) - 1


def mix64(z):
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def u01(key, it, k):
    return (mix64(key ^ (4 * it + k)) >> 11) * 2.0 ** -53


def exact_sdf(prims, verts, x, y):
    best = math.inf
    for q in prims:
        if q["type"] == _abi.OBS_CIRCLE:
            dx, dy = x - q["cx"], y - q["cy"]
            v = math.sqrt(dx * dx + dy * dy) - (q["size"] + q["margin"])
        elif q["type"] == _abi.OBS_SQUARE:
            half = q["size"] / 2 + q["margin"]
            dx, dy = abs(x - q["cx"]) - half, abs(y - q["cy"]) - half
            ox, oy = max(dx, 0.0), max(dy, 0.0)
            v = math.sqrt(ox * ox + oy * oy) + min(max(dx, dy), 0.0)
        else:
            V = verts[q["v0"]:q["v0"] + q["nv"]]
            d, inside = math.inf, False
            for e in range(len(V)):
                (x0, y0), (x1, y1) = V[e], V[(e + 1) % len(V)]
                ex, ey = x1 - x0, y1 - y0
                t = ((x - x0) * ex + (y - y0) * ey) / (ex * ex + ey * ey)
                t = min(max(t, 0.0), 1.0)
                qx, qy = x - (x0 + t * ex), y - (y0 + t * ey)
                d = min(d, math.sqrt(qx * qx + qy * qy))
                if (y0 > y) != (y1 > y) and x < x0 + (y - y0) * ex / (y1 - y0):
                    inside = not inside
            v = (-d if inside else d) - q["margin"]
        best = min(best, v)
    return best


def inflation(problem, margin):
    """trajectory_initialization.py:108-113 (RectangleGeometry: max |np.min(point)| + margin; else 0)."""
    if problem.shape != "rectangle":
        return 0.0
    return max(abs(min(pt)) for pt in problem.body) + margin


def linspace_at(a, b, num, i):
    if num == 1:
        return a
    if i == num - 1:
        return b
    return i * ((b - a) / (num - 1)) + a


def rrt_one(problem, x0, xg, bounds, step_size=0.05, max_iter=1000, margin=0.01, goal_sample_rate=0.05, seed=0,
            instance=0):
    """-> (X_init [N+1, nx], ok).  Mirrors _build_rrt_path; ok = False where the reference raises."""
    prims, verts = expand(problem.obstacles)
    sdf = lambda x, y: exact_sdf(prims, verts, x, y)  # noqa: E731
    infl = inflation(problem, margin)
    npts, nx = problem.N + 1, problem.nx
    (bx0, by0), (bx1, by1) = bounds
    key = mix64((seed & M64) ^ mix64(instance))

    def free(p1, p2):
        dx, dy = p2[0] - p1[0], p2[1] - p1[1]
        n = max(1, int(math.ceil(math.sqrt(dx * dx + dy * dy) / step_size)))
        return all(sdf(p1[0] + dx * (i / n), p1[1] + dy * (i / n)) >= infl for i in range(n + 1))

    sx, sy, gx, gy = float(x0[0]), float(x0[1]), float(xg[0]), float(xg[1])
    nodes, parent, final = [(sx, sy)], [-1], None
    for it in range(max_iter):
        if u01(key, it, 0) < goal_sample_rate:
            rx, ry = gx, gy
        else:
            rx, ry = bx0 + (bx1 - bx0) * u01(key, it, 1), by0 + (by1 - by0) * u01(key, it, 2)
        d = [math.sqrt((rx - a) * (rx - a) + (ry - b) * (ry - b)) for a, b in nodes]
        k = int(np.argmin(d))
        ax, ay = nodes[k]
        dx, dy = rx - ax, ry - ay
        nrm = math.sqrt(dx * dx + dy * dy)
        if nrm == 0:
            continue
        qx, qy = ax + (dx / nrm) * step_size, ay + (dy / nrm) * step_size
        if free((ax, ay), (qx, qy)):
            nodes.append((qx, qy))
            parent.append(k)
            ex, ey = qx - gx, qy - gy
            if math.sqrt(ex * ex + ey * ey) < step_size:
                final = len(nodes) - 1
                break
    if final is None:
        return np.array([[linspace_at(x0[c], xg[c], npts, k) for c in range(nx)] for k in range(npts)]), False
    path = [(gx, gy)]
    j = final
    while j >= 0:
        path.append(nodes[j])
        j = parent[j]
    path = np.array(path[::-1])
    # insert_intermediate_points (max_angle_deg 60)
    pts = [path[0]]
    for i in range(1, len(path) - 1):
        v1, v2 = path[i] - path[i - 1], path[i + 1] - path[i]
        c = (v1[0] * v2[0] + v1[1] * v2[1]) / (math.sqrt(v1[0] ** 2 + v1[1] ** 2) * math.sqrt(v2[0] ** 2 + v2[1] ** 2))
        if math.acos(min(max(c, -1.0), 1.0)) * 57.29577951308232 > 60:
            pts.append((path[i] + path[i - 1]) / 2)
        pts.append(path[i])
    pts.append(path[-1])
    pts = np.array(pts)
    # _shortcut_path
    new, i = [pts[0]], 0
    while i < len(pts) - 1:
        j = len(pts) - 1
        while j > i + 1:
            if free(pts[i], pts[j]):
                break
            j -= 1
        new.append(pts[j])
        i = j
    pts = np.array(new)
    # _bspline_curve
    if len(pts) <= 2:
        xy = np.linspace(pts[0], pts[-1], npts)
    else:
        s = np.linspace(0, 1, len(pts))
        s_new = np.linspace(0, 1, npts)
        xy = np.vstack((CubicSpline(s, pts[:, 0])(s_new), CubicSpline(s, pts[:, 1])(s_new))).T
    X = np.zeros((npts, nx))
    X[:, 0:2] = xy
    return X, True
