"""The oracle's NLP building blocks against golden vectors computed by the REFERENCE's own code
(tests/golden/nlp_golden.json, made by tests/golden/make_nlp_golden.py under a numeric casadi stub):
dynamics of all 6 models, rectangle/triangle corners, soft_min, the analytic obstacle SDFs, and the
Config parses of the 6 shipped benchmarks."""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "nlp_golden.json")))


def test_dynamics_all_six_models():
    import oracle as O
    from nlotrajectories_amd.problem import Problem

    seen = set()
    for rec in GOLD["dynamics"]:
        name = rec["dynamics"]
        seen.add(name)
        kw = dict(dynamics=name, shape="dot")
        if rec["wheelbase"] is not None:
            kw["wheelbase"] = rec["wheelbase"]
        p = Problem(**kw, obstacles=[{"type": "circle", "center": (0, 0), "radius": 0.1}])
        f = O.dynamics(p, rec["x"], rec["u"])
        np.testing.assert_allclose(f, rec["f"], rtol=1e-13, atol=1e-13, err_msg=str(rec))
    assert seen == {"point_1st", "point_2nd", "unicycle", "unicycle_2nd", "ackermann", "ackermann_2nd"}


def test_corners_rectangle_and_triangle():
    import oracle as O
    from nlotrajectories_amd.problem import Problem

    for rec in GOLD["corners"]:
        p = Problem(shape=rec["shape"], length=rec["length"], width=rec["width"],
                    obstacles=[{"type": "circle", "center": (0, 0), "radius": 0.1}])
        c = O.corners(p, rec["pose"] + [0.0, 0.0])
        np.testing.assert_allclose(c, rec["corners"], rtol=0, atol=1e-14)


def test_soft_min():
    import oracle as O

    for rec in GOLD["soft_min"]:
        assert abs(O.soft_min(rec["v"]) - rec["soft_min"]) <= 1e-14 * max(1.0, abs(rec["soft_min"]))


SCENES = ["benchmark_1_dot_circle.yaml", "benchmark_2_unicycle_circle.yaml", "benchmark_3_unicycle_convex.yaml",
          "benchmark_4_dot_nonconvex.yaml", "benchmark_5_ackermann_circle.yaml", "benchmark_6_ackermann_wave.yaml"]


@pytest.mark.parametrize("fn", SCENES)
def test_scene_sdf_circle_square(fn):
    """MultiObstacle.approximated_sdf of the six benchmark scenes (circles, squares, benchmark_4's polygon,
    benchmark_6's elliptical rings) through the YAML -> Problem mapping."""
    import oracle as O
    from nlotrajectories_amd.config import Config

    cfg = Config.model_validate(GOLD["configs"][fn])
    prob = cfg.to_problem().with_(sdf="analytic")
    pts = np.asarray(GOLD["sdf"]["points"])
    v = O.sdf_eval(prob, pts)[:, 0]
    np.testing.assert_allclose(v, GOLD["scene_sdf"][fn], rtol=0, atol=1e-12)


def test_configs_parse_like_reference():
    """Our schema accepts each reference Config dump and reproduces it field for field."""
    from nlotrajectories_amd.config import Config

    assert len(GOLD["configs"]) == 6
    for fn, ref in GOLD["configs"].items():
        ours = json.loads(Config.model_validate(ref).model_dump_json())
        assert ours["body"] == ref["body"], fn
        assert ours["solver"]["N"] == ref["solver"]["N"] and ours["solver"]["dt"] == ref["solver"]["dt"], fn
        for k in ("use_slack", "slack_penalty", "use_smooth", "smooth_weight", "mode", "type"):
            assert ours["solver"][k] == ref["solver"][k], (fn, k)
        assert ours["model"] == ref["model"], fn
        assert ours["obstacles"] == ref["obstacles"], fn


# the single obstacles of make_nlp_golden.py (casadi.py constructors with those arguments), as scene dicts
SINGLE = {
    "circle": {"type": "circle", "center": (0.5, 0.5), "radius": 0.2, "margin": 0.05},
    "square": {"type": "square", "center": (0.8, 0.2), "size": 0.35, "margin": 0.01},
    "polygon": {"type": "polygon", "points": [(0.1, 0.1), (0.6, 0.15), (0.7, 0.6), (0.2, 0.5)], "margin": 0.02},
    "elliptical_ring": {"type": "elliptical_ring", "center": (0.25, 0.2), "semi_axes": (0.25, 0.2), "width": 0.05,
                        "angle": 3.14, "margin": 0.01},
    "elliptical_ring_neg": {"type": "elliptical_ring", "center": (0.7, 0.2), "semi_axes": (0.25, 0.2), "width": 0.05,
                            "angle": -3.14, "margin": 0.01},
    "trapezoid": {"type": "trapezoid", "points": [(0.2, 0.2), (0.8, 0.2), (0.6, 0.6), (0.4, 0.6)], "margin": 0.01},
    "convex_elliptic_ring": {"type": "convex_elliptic_ring", "center": (0.5, 0.4), "semi_axes": (0.3, 0.25),
                             "width": 0.06, "angle": 3.0, "num_arc_points": 8, "margin": 0.01, "rotation": 0.3},
    "discr_s": {"type": "discr_s", "center": (0.3, 0.5), "semi_axes": (0.25, 0.2), "width": 0.05, "angle": 3.14,
                "num_arc_points": 10, "margin": 0.01},
}


@pytest.mark.parametrize("name", list(SINGLE))
def test_single_obstacle_sdf(name):
    """approximated_sdf of each analytic obstacle type (the golden vectors record the obstacle alone; the
    scene wraps it in a one-term soft_min, which is the identity: -1/a log(exp(-a v)) = v to rounding)."""
    import oracle as O
    from nlotrajectories_amd.problem import Problem

    prob = Problem(shape="dot", dynamics="point_2nd", obstacles=[SINGLE[name]])
    pts = np.asarray(GOLD["sdf"]["points"])
    v = O.sdf_eval(prob, pts)[:, 0]
    np.testing.assert_allclose(v, GOLD["sdf"][name], rtol=0, atol=1e-12, err_msg=name)


@pytest.mark.parametrize("name", ["polygon", "trapezoid", "discr_s", "elliptical_ring"])
def test_analytic_sdf_derivatives_match_finite_differences(name):
    """The oracle's gradient / Hessian of the scene SDF (what the solver uses) against central differences."""
    import oracle as O
    from nlotrajectories_amd.problem import Problem

    prob = Problem(shape="dot", dynamics="point_2nd", obstacles=[SINGLE[name]])
    rng = np.random.default_rng(5)
    P = rng.uniform(-0.3, 1.3, size=(40, 2))
    h = 1e-6
    out = O.sdf_eval(prob, P)
    for a in range(2):
        e = np.zeros(2)
        e[a] = h
        fp, fm = O.sdf_eval(prob, P + e), O.sdf_eval(prob, P - e)
        g_fd = (fp[:, 0] - fm[:, 0]) / (2 * h)
        np.testing.assert_allclose(out[:, 1 + a], g_fd, rtol=1e-5, atol=1e-6, err_msg=(name, a))
        # Hessian row a from differences of the gradient (xx, xy, yy at columns 3, 4, 5)
        H_fd = (fp[:, 1:3] - fm[:, 1:3]) / (2 * h)
        cols = (3, 4) if a == 0 else (4, 5)
        np.testing.assert_allclose(out[:, cols], H_fd, rtol=1e-4, atol=1e-4, err_msg=(name, a))


@pytest.mark.parametrize("dyn", ["point_1st", "point_2nd", "unicycle", "unicycle_2nd", "ackermann", "ackermann_2nd"])
def test_rk4_defect_map(dyn):
    """The opt-in RK4 defect map (integrator='rk4'; not the reference's Euler NLP) equals the classical RK4 step
    of the reference's own f (golden-pinned above), and its A, B match central differences."""
    import oracle as O
    from nlotrajectories_amd.problem import Problem

    kw = dict(dynamics=dyn, shape="dot", dt=0.1, obstacles=[{"type": "circle", "center": (0, 0), "radius": 0.1}])
    if "ackermann" in dyn:
        kw["wheelbase"] = 0.1
    p = Problem(**kw).with_(integrator="rk4")
    rng = np.random.default_rng(2)
    x, u = rng.uniform(-0.8, 0.8, p.nx), rng.uniform(-1, 1, p.nu)
    f = lambda z: np.asarray(O.dynamics(p, z, u))  # noqa: E731
    k1 = f(x)
    k2 = f(x + 0.5 * p.dt * k1)
    k3 = f(x + 0.5 * p.dt * k2)
    k4 = f(x + p.dt * k3)
    F, A, B = O.dyn_map(p, x, u)
    np.testing.assert_allclose(F, x + p.dt * (k1 + 2 * k2 + 2 * k3 + k4) / 6, rtol=0, atol=1e-14)
    h = 1e-6
    for j in range(p.nx):
        e = np.zeros(p.nx)
        e[j] = h
        np.testing.assert_allclose(A[:, j], (O.dyn_map(p, x + e, u)[0] - O.dyn_map(p, x - e, u)[0]) / (2 * h), atol=1e-7)
    for j in range(p.nu):
        e = np.zeros(p.nu)
        e[j] = h
        np.testing.assert_allclose(B[:, j], (O.dyn_map(p, x, u + e)[0] - O.dyn_map(p, x, u - e)[0]) / (2 * h), atol=1e-7)
    Fe, _, _ = O.dyn_map(p.with_(integrator="euler"), x, u)
    np.testing.assert_allclose(Fe, x + p.dt * k1, atol=1e-15)
