"""Golden vectors of the NLP building blocks, computed by the REFERENCE's own code (run only where
/root/reference exists; the output tests/golden/nlp_golden.json is what travels).

The reference's expression code (core/dynamics.py, geometry.py, utils.py, sdf/casadi.py, config.py) only
needs `casadi` for symbolic arithmetic, `shapely` for exact polygon distances and `matplotlib` for
drawing.  SURVEY.md §8c: with a NUMERIC casadi stub (MX = float64 ndarray, cos/sin/... = numpy,
vertcat = stacking), data-holder shapely/matplotlib stubs and an empty l4casadi, the reference modules
import and evaluate numerically.  The stubs are written to a temporary directory (never into the repo)
and put ahead of the reference's src/ on sys.path for this process only.

Recorded (all inputs seeded, numpy PCG64):
  * dynamics f(x, u) of the 6 models (core/dynamics.py:33-148), Ackermann wheelbases 0.1 / 0.05 / 1.0;
  * footprint corners of RectangleGeometry / TriangleGeometry (core/geometry.py:78-83,125-144);
  * soft_min (core/utils.py:18-33) of seeded vectors;
  * approximated_sdf of Circle, Square, Polygon, EllipticRing, Trapezoid, ConvexEllipticRing, ConvexSObstacle
    and of the MultiObstacle scenes of benchmarks 1-6 (core/sdf/casadi.py:27-525);
  * Config(**yaml) of benchmarks 1-6 (core/config.py:215-222), model_dump'ed.

    python tests/golden/make_nlp_golden.py [--reference /root/reference]
"""
import argparse
import json
import os
import sys
import tempfile
import textwrap

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

STUBS = {
    "casadi/__init__.py": '''
        import numpy as _np
        class MX(_np.ndarray):
            def __new__(cls, v=0.0):
                return _np.asarray(v, dtype=_np.float64).view(cls)
        SX = MX
        class Opti:  # the NLP container is not used by the recorded functions
            pass
        cos, sin, tan, tanh, exp, log, sqrt = _np.cos, _np.sin, _np.tan, _np.tanh, _np.exp, _np.log, _np.sqrt
        fmax, fmin = _np.maximum, _np.minimum
        def vertcat(*a):
            return _np.concatenate([_np.atleast_1d(_np.asarray(x, dtype=_np.float64)) for x in a])
        def hcat(a):
            return _np.concatenate([_np.asarray(x).reshape(-1, 1) for x in a], axis=1)
        def reshape(a, r, c):
            return _np.asarray(a).reshape(r, c)
        def sum1(a):
            return _np.sum(a, axis=0)
        def sum2(a):
            return _np.sum(a, axis=1, keepdims=True)
    ''',
    "shapely/__init__.py": "",
    "shapely/geometry.py": '''
        class Point:
            def __init__(self, *a): self.coords = a
        class Polygon:
            def __init__(self, pts): self.points = pts
    ''',
    "matplotlib/__init__.py": "",
    "matplotlib/patches.py": '''
        class _Patch:
            def __init__(self, *a, **k): pass
        Circle = Rectangle = Polygon = _Patch
    ''',
    "matplotlib/axes/__init__.py": "",
    "matplotlib/axes/_axes.py": "class Axes: pass\n",
    "l4casadi/__init__.py": "",
}


def write_stubs(d):
    for rel, src in STUBS.items():
        p = os.path.join(d, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(textwrap.dedent(src))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(HERE, "nlp_golden.json"))
    a = ap.parse_args()
    stub_dir = tempfile.mkdtemp(prefix="nlot_casadi_stub_")
    write_stubs(stub_dir)
    sys.path[:0] = [stub_dir, os.path.join(a.reference, "src")]
    import yaml
    from nlotrajectories.core import dynamics as D
    from nlotrajectories.core import geometry as G
    from nlotrajectories.core import utils as U
    from nlotrajectories.core.config import Config
    from nlotrajectories.core.sdf import casadi as S

    rng = np.random.default_rng(20260101)
    out = {"generator": "tests/golden/make_nlp_golden.py (reference code under a numeric casadi stub)"}

    # ---- dynamics ----
    dyn = []
    for name, cls in D.DYNAMICS_CLASS_MAP.items():
        for L in ((0.1, 0.05, 1.0) if "ackermann" in name.value else (None,)):
            m = cls(L) if L is not None else cls()
            nx, nu = m.state_dim(), m.control_dim()
            for _ in range(6):
                x = rng.uniform(-1.2, 1.2, nx)
                u = rng.uniform(-1.5, 1.5, nu)
                f = np.asarray(m.dynamics(x, u), dtype=np.float64).ravel()
                dyn.append({"dynamics": name.value, "wheelbase": L, "x": x.tolist(), "u": u.tolist(), "f": f.tolist()})
    out["dynamics"] = dyn

    # ---- corners ----
    corners = []
    for shape, cls in (("rectangle", G.RectangleGeometry), ("triangle", G.TriangleGeometry)):
        for (length, width) in ((0.2, 0.1), (0.2, 0.08), (0.1, 0.1), (0.08, 0.05)):
            g = cls(length, width)
            for _ in range(4):
                pose = np.array([rng.uniform(-1, 2), rng.uniform(-1, 2), rng.uniform(-np.pi, np.pi)])
                pts = [(float(np.asarray(px)), float(np.asarray(py))) for px, py in g.transform(pose)]
                corners.append({"shape": shape, "length": length, "width": width, "pose": pose.tolist(),
                                "corners": pts})
    out["corners"] = corners

    # ---- soft_min ----
    sm = []
    for n in (1, 2, 3, 4, 7):
        for _ in range(3):
            v = rng.uniform(-0.5, 1.0, n)
            sm.append({"v": v.tolist(), "soft_min": float(np.asarray(U.soft_min([np.array([t]) for t in v])).ravel()[0])})
    out["soft_min"] = sm

    # ---- analytic approximated SDFs ----
    P = rng.uniform(-0.6, 1.6, size=(64, 2))
    xs, ys = P[:, 0].copy(), P[:, 1].copy()
    obstacles = {
        "circle": S.CircleObstacle((0.5, 0.5), 0.2, 0.05),
        "square": S.SquareObstacle((0.8, 0.2), 0.35, 0.01),
        "polygon": S.PolygonObstacle([(0.1, 0.1), (0.6, 0.15), (0.7, 0.6), (0.2, 0.5)], 0.02),
        "elliptical_ring": S.EllipticRingObstacle((0.25, 0.2), (0.25, 0.2), 0.05, angle=3.14, margin=0.01),
        "elliptical_ring_neg": S.EllipticRingObstacle((0.7, 0.2), (0.25, 0.2), 0.05, angle=-3.14, margin=0.01),
        "trapezoid": S.TrapezoidObstacle([(0.2, 0.2), (0.8, 0.2), (0.6, 0.6), (0.4, 0.6)], 0.01),
        "convex_elliptic_ring": S.ConvexEllipticRing((0.5, 0.4), (0.3, 0.25), 0.06, angle=3.0, num_arc_points=8,
                                                     margin=0.01, rotation=0.3),
        "discr_s": S.ConvexSObstacle((0.3, 0.5), (0.25, 0.2), 0.05, angle=3.14, num_arc_points=10, margin=0.01),
    }
    sdfs = {"points": P.tolist()}
    for k, o in obstacles.items():
        sdfs[k] = np.asarray(o.approximated_sdf(xs, ys), dtype=np.float64).ravel().tolist()
    out["sdf"] = sdfs

    # ---- benchmark configs and their scenes ----
    bdir = os.path.join(a.reference, "src", "nlotrajectories", "benchmarks")
    cfgs, scenes = {}, {}
    for fn in sorted(os.listdir(bdir)):
        if not fn.endswith(".yaml"):
            continue
        with open(os.path.join(bdir, fn)) as f:
            c = Config(**yaml.safe_load(f))
        cfgs[fn] = json.loads(c.model_dump_json())
        scene = c.get_obstacles()
        scenes[fn] = np.asarray(scene.approximated_sdf(xs, ys), dtype=np.float64).ravel().tolist()
    out["configs"] = cfgs
    out["scene_sdf"] = scenes

    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", a.out, {k: len(v) for k, v in out.items() if isinstance(v, (list, dict))})


if __name__ == "__main__":
    main()
