"""Analytic obstacle scenes -> the primitive obstacles and vertex pool of `NlotProblem` (include/nlot.h).

The reference builds its scene objects in core/sdf/casadi.py; their approximated_sdf evaluates four
primitive formulas, which the GPU kernels (nlot_device.h) and the oracle (oracle/nlot_oracle.c) restate:

    circle     CircleObstacle       casadi.py:27-45
    square     SquareObstacle       casadi.py:48-118
    polygon    PolygonObstacle      casadi.py:127-186   (also EllipticRingObstacle, casadi.py:193-248)
    trapezoid  TrapezoidObstacle    casadi.py:251-374   (also the pieces of ConvexEllipticRing / ConvexSObstacle)

The composite obstacles are generated here exactly as their constructors do (same numpy calls in the same
order, so the vertices are bitwise the reference's): an elliptical ring becomes one polygon of its 2n arc
points; a convex elliptic ring (casadi.py:393-445) and a discr_s (ConvexSObstacle, casadi.py:448-525) become a
*group* of trapezoids, soft_min'ed among themselves first (they are MultiObstacles nested in the scene's
MultiObstacle, casadi.py:385-386).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

from . import _abi


def _ring_points(center, semi_axes, width, angle, num_arc_points, rotation):
    """EllipticRingObstacle.__init__ (casadi.py:217-246): outer arc, then the inner arc reversed, rotated and
    translated."""
    center = np.array(center)
    outer_a, outer_b = semi_axes
    inner_a, inner_b = outer_a - width, outer_b - width
    if inner_a <= 0 or inner_b <= 0:
        raise ValueError("Width too large for given semi-axes.")
    cx, cy = center
    t = np.linspace(0.0, angle, num_arc_points)
    outer = [(outer_a * np.cos(ti), outer_b * np.sin(ti)) for ti in t]
    inner = [(inner_a * np.cos(ti), inner_b * np.sin(ti)) for ti in t[::-1]]
    return [(cx + (x * np.cos(rotation) - y * np.sin(rotation)), cy + (x * np.sin(rotation) + y * np.cos(rotation)))
            for x, y in outer + inner]


def _arc_quads(cx, cy, outer_a, outer_b, inner_a, inner_b, t, rotation, reverse):
    """The quads between corresponding outer / inner arc samples (casadi.py:416-442, 471-522)."""
    outer_raw = [(outer_a * np.cos(ti), outer_b * np.sin(ti)) for ti in t]
    inner_raw = [(inner_a * np.cos(ti), inner_b * np.sin(ti)) for ti in t]
    cos_r, sin_r = np.cos(rotation), np.sin(rotation)

    def transform(pt):
        x, y = pt
        return (x * cos_r - y * sin_r + cx, x * sin_r + y * cos_r + cy)

    outer_pts = [transform(p) for p in outer_raw]
    inner_pts = [transform(p) for p in inner_raw]
    quads = []
    for i in range(len(t) - 1):
        q = [outer_pts[i], outer_pts[i + 1], inner_pts[i + 1], inner_pts[i]]
        quads.append(q[::-1] if reverse else q)
    return quads


def _convex_ring_quads(center, semi_axes, width, angle, num_arc_points, rotation, s_shape):
    cx, cy = center
    outer_a, outer_b = semi_axes
    inner_a, inner_b = outer_a - width, outer_b - width
    if inner_a <= 0 or inner_b <= 0:
        raise ValueError("Width too large for given semi-axes.")
    quads = _arc_quads(cx, cy, outer_a, outer_b, inner_a, inner_b, np.linspace(0.0, angle, num_arc_points), rotation,
                       False)
    if s_shape:  # ConvexSObstacle's second half: shifted by 0.45 in x, the arc mirrored, vertex order reversed
        quads += _arc_quads(cx + 0.45, cy, outer_a, outer_b, inner_a, inner_b,
                            np.linspace(0.0, -angle, num_arc_points), rotation, True)
    return quads


def expand(obstacles) -> Tuple[List[dict], List[Tuple[float, float]]]:
    """Scene obstacle dicts (the reference's YAML vocabulary, core/config.py:53-142, plus
    "convex_elliptic_ring") -> (primitives, vertices).  A primitive is a dict with type (an _abi.OBS_* code),
    group, v0, nv, cx, cy, size, margin."""
    prims, verts = [], []
    group = 0

    def poly(points, margin, kind, grp):
        pts = [(float(x), float(y)) for x, y in points]
        if kind == _abi.OBS_TRAPEZOID and len(pts) != 4:
            raise ValueError("TrapezoidObstacle requires exactly 4 vertices.")
        c = np.mean(points, axis=0) if kind == _abi.OBS_POLYGON else (0.0, 0.0)  # casadi.py:133
        prims.append(dict(type=kind, group=grp, v0=len(verts), nv=len(pts), cx=float(c[0]), cy=float(c[1]), size=0.0,
                          margin=float(margin)))
        verts.extend(pts)

    for o in obstacles:
        t = o["type"]
        m = float(o.get("margin", 0.0))
        if t == "circle":
            prims.append(dict(type=_abi.OBS_CIRCLE, group=-1, v0=0, nv=0, cx=float(o["center"][0]),
                              cy=float(o["center"][1]), size=float(o["radius"]), margin=m))
        elif t == "square":
            prims.append(dict(type=_abi.OBS_SQUARE, group=-1, v0=0, nv=0, cx=float(o["center"][0]),
                              cy=float(o["center"][1]), size=float(o["size"]), margin=m))
        elif t == "polygon":
            poly(o["points"], m, _abi.OBS_POLYGON, -1)
        elif t == "trapezoid":
            poly(o["points"], m, _abi.OBS_TRAPEZOID, -1)
        elif t == "elliptical_ring":
            poly(_ring_points(o["center"], o["semi_axes"], o["width"], o.get("angle", np.pi),
                              o.get("num_arc_points", 15), o.get("rotation", 0.0)), m, _abi.OBS_POLYGON, -1)
        elif t in ("convex_elliptic_ring", "discr_s"):
            quads = _convex_ring_quads(o["center"], o["semi_axes"], o["width"], o.get("angle", np.pi),
                                       o.get("num_arc_points", 15 if t == "convex_elliptic_ring" else 30),
                                       o.get("rotation", 0.0), t == "discr_s")
            for q in quads:
                poly(q, m, _abi.OBS_TRAPEZOID, group)
            group += 1
        else:
            raise ValueError(f"unknown obstacle type {t!r}")
    if len(prims) > _abi.MAX_OBS:
        raise ValueError(f"scene expands to {len(prims)} primitive obstacles (at most {_abi.MAX_OBS})")
    if len(verts) > _abi.MAX_VERTS:
        raise ValueError(f"scene has {len(verts)} vertices (at most {_abi.MAX_VERTS})")
    return prims, verts
