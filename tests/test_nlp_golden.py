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
          "benchmark_5_ackermann_circle.yaml"]


@pytest.mark.parametrize("fn", SCENES)
def test_scene_sdf_circle_square(fn):
    """MultiObstacle.approximated_sdf of the circle/square scenes through the YAML -> Problem mapping."""
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
