"""YAML surface: the schema (config.py) validates the shipped scenario files and maps them onto the same
NLP as the restated BENCHMARKS; the reference's malformed configs/*.yaml are rejected;
the CLI fails loudly on what is not built (sqpmethod, learned SDF without weights)."""
import glob
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CFG = os.path.join(HERE, "golden", "configs")
REF = "/root/reference/src/nlotrajectories/benchmarks"


def test_restated_configs_map_to_benchmarks():
    from nlotrajectories_amd.config import Config
    from nlotrajectories_amd.problem import BENCHMARKS

    for key, name in (("b1", "benchmark_1_dot_circle"), ("b2", "benchmark_2_unicycle_circle"),
                      ("b5", "benchmark_5_ackermann_circle")):
        p = Config.load(os.path.join(CFG, name + ".yaml")).to_problem()
        q = BENCHMARKS[key]["problem"]
        for f in ("dynamics", "shape", "N", "dt", "use_slack", "slack_penalty", "enforce_heading", "sdf"):
            assert getattr(p, f) == getattr(q, f), (name, f)
        assert np.allclose(p.control_bounds, q.control_bounds)
        assert [o["type"] for o in p.obstacles] == [o["type"] for o in q.obstacles]
        assert bytes(p.to_c()) == bytes(q.to_c())


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present (GPU box)")
def test_reference_yaml_files_validate():
    from nlotrajectories_amd.config import Config

    files = sorted(glob.glob(os.path.join(REF, "*.yaml")))
    assert len(files) == 6
    for f in files:
        c = Config.load(f)
        assert c.solver.type == "ipopt" and c.solver.initializer.choice.mode == "rrt"
        c.to_problem()
    for f in sorted(glob.glob("/root/reference/configs/*.yaml")):
        with pytest.raises(Exception):
            Config.load(f)


def test_cli_refuses_what_is_not_built(tmp_path):
    import yaml

    from nlotrajectories_amd.cli import run_benchmark

    base = yaml.safe_load(open(os.path.join(CFG, "benchmark_2_unicycle_circle.yaml")))
    f = tmp_path / "sqp.yaml"
    base["solver"]["type"] = "sqpmethod"
    f.write_text(yaml.safe_dump(base))
    with pytest.raises(NotImplementedError, match="sqpmethod"):
        run_benchmark(f, initializer="linear")


def test_scene_metrics_against_exact():
    from nlotrajectories_amd import scene

    obs = [{"type": "circle", "center": (0.5, 0.5), "radius": 0.2, "margin": 0.05},
           {"type": "square", "center": (1.2, 0.4), "size": 0.3, "margin": 0.0}]
    x = np.linspace(-1, 2, 301)
    X, Y = np.meshgrid(x, x)
    ex = scene.exact_sdf(obs, X, Y)
    ap = scene.approximated_sdf(obs, X, Y)
    assert abs(ex[150, 50] - (np.hypot(0.5 - 0.5, 0.5 - 0.5) - 0.25)) < 1e-12 or ex.min() < 0
    assert scene.iou(ex, ap) > 0.9 and scene.mse(ex, ap) < 1e-3
    assert scene.hausdorff(ex, ex, X, Y) == 0.0 and scene.chamfer(ex, ex, X, Y) == 0.0
