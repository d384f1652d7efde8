"""The learned-SDF trainer restatement (core/sdf/l4casadi.py:14-228) on the CPU: sampling, targets from the
exact scene SDF, the loss terms, early stopping, and that the result is consumable by the SDF kernels."""
import json
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def _b6():
    from nlotrajectories_amd.config import Config

    g = json.load(open(os.path.join(HERE, "golden", "nlp_golden.json")))
    return Config.model_validate(g["configs"]["benchmark_6_ackermann_wave.yaml"])


def test_sample_points_boundary_share_and_band():
    from nlotrajectories_amd import scene
    from nlotrajectories_amd.trainer import sample_points

    cfg = _b6()
    sdf = lambda x, y: scene.exact_sdf(cfg.obstacle_dicts(), x, y)  # noqa: E731
    xs, ys = sample_points((-0.5, 1.5), (-0.5, 1.5), 10000, sdf, margin=0.05, boundary_fraction=0.3,
                           rng=np.random.default_rng(1))
    assert len(xs) == 10000
    tail = sdf(xs[7000:], ys[7000:])
    assert np.abs(tail).max() < 0.05  # the boundary-focused share lies in the band


def test_exact_scene_sdf_of_rings_and_polygon():
    """Exact SDF (PolygonObstacle.sdf: boundary distance signed by containment) at points with known answers."""
    from nlotrajectories_amd import scene

    sq = [{"type": "polygon", "points": [(0, 0), (1, 0), (1, 1), (0, 1)], "margin": 0.0}]
    v = scene.exact_sdf(sq, np.array([0.5, 1.5, 0.5]), np.array([0.5, 0.5, 0.9]))
    np.testing.assert_allclose(v, [-0.5, 0.5, -0.1], atol=1e-12)
    cfg = _b6()
    # a point inside the first ring's band (outer radius 0.25 x 0.2 about (0.25, 0.2), width 0.05): negative
    assert scene.exact_sdf(cfg.obstacle_dicts(), np.array([0.25]), np.array([0.2 + 0.175]))[0] < 0
    assert scene.exact_sdf(cfg.obstacle_dicts(), np.array([0.25]), np.array([0.2]))[0] > 0  # the ring's hollow


def test_trainer_reduces_loss_and_feeds_the_kernels():
    from nlotrajectories_amd.nn import MlpWeights
    from nlotrajectories_amd.trainer import NNObstacleTrainer, model_from_config

    cfg = _b6()
    torch.manual_seed(0)
    tr = NNObstacleTrainer(cfg.obstacle_dicts(), model_from_config(cfg.model), device="cpu", epochs=2,
                           n_samples=6000, boundary_fraction=cfg.model.boundary_fraction,
                           eikonal_weight=cfg.model.eikonal_loss_weight,
                           surface_loss_weight=cfg.model.surface_loss_weight, seed=0, verbose=False)
    tr.train((-0.5, 1.5), (-0.5, 1.5))
    assert tr.history[-1][1] < tr.history[0][1] or len(tr.history) == 1
    w = MlpWeights.from_module(tr.model)
    assert w.hidden == 128 and w.n_hidden == 1  # MultiLayerPerceptron(2, 128, 1, 2): one HxH layer
    # deterministic: same seed, same first-epoch losses
    tr2 = NNObstacleTrainer(cfg.obstacle_dicts(), model_from_config(cfg.model), device="cpu", epochs=1,
                            n_samples=6000, boundary_fraction=cfg.model.boundary_fraction,
                            eikonal_weight=cfg.model.eikonal_loss_weight,
                            surface_loss_weight=cfg.model.surface_loss_weight, seed=0, verbose=False)
    tr2.train((-0.5, 1.5), (-0.5, 1.5))
    assert abs(tr2.history[0][0] - tr.history[0][0]) < 1e-6


def test_restated_b4_b6_equal_their_yaml():
    """problem.BENCHMARKS b4 / b6 (restated so the GPU box can build them) equal the reference's YAML dumps
    byte for byte in the C struct."""
    from nlotrajectories_amd.config import Config
    from nlotrajectories_amd.problem import BENCHMARKS

    g = json.load(open(os.path.join(HERE, "golden", "nlp_golden.json")))
    for k, fn in (("b4", "benchmark_4_dot_nonconvex.yaml"), ("b6", "benchmark_6_ackermann_wave.yaml")):
        c = Config.model_validate(g["configs"][fn])
        a = BENCHMARKS[k]["problem"].with_(sdf="analytic").to_c()
        b = c.to_problem().with_(sdf="analytic").to_c()
        assert bytes(a) == bytes(b), k
        assert BENCHMARKS[k]["start"] == list(c.body.start_state) and BENCHMARKS[k]["goal"] == list(c.body.goal_state)
